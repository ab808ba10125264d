set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
# SQ counters of the decode kernels (one pass, <= 8 SQ counters, kernel trace only)
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/pmcsq -o run -- python3 tools/bench_decode.py > gpurun_out/pmcsq.log 2>&1 || { tail -5 gpurun_out/pmcsq.log; exit 1; }
python - <<'PY'
import csv, collections, re
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open("gpurun_out/pmcsq/run_counter_collection.csv")):
    k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("swh::(anonymous namespace)::", ""))
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = open("gpurun_out/r3_sq_pmc_decode.txt", "w")
for k, cs in agg.items():
    if not any(s in k for s in ("lm_head", "xstream", "attn_decode")):
        continue
    line = k[:60] + "  " + "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(cs.items()))
    print(line); out.write(line + "\n")
PY
rm -rf gpurun_out/pmcsq
