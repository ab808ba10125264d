"""Per-launch HBM traffic of the decode kernels from two rocprofv3 PMC passes
(`--pmc FETCH_SIZE`, `--pmc WRITE_SIZE`, each with --kernel-trace only) of
tools/bench_decode.py, corrected as MI355X_MICROARCH.md §HBM prescribes:
FETCH_SIZE counts half the bytes of wide streaming reads on gfx950 (x2);
both counters are KiB.  Writes profiles/<name>.json, which bench.py reads
for `roofline.traffic`.

    python tools/pmc_summary.py gpurun_out/pmcf gpurun_out/pmcw profiles/r2_pmc_decode.json [source script]
"""
import collections
import csv
import json
import re
import sys

NAMES = {  # kernel template prefix -> the bench's kernel name
    "lm_head_kernel<2, 2, false, false": "decode_gemm.gate_up",   # tile kernel, folded norm, SiLU epilogue
    "lm_head_kernel<2, 2, false, 0": "decode_gemm.gate_up",       # (round 4: SAMPLE is an int)
    "decode_gemm_kernel<1, 2, 2, 0, true": "decode_gemm.qkv",
    "decode_gemm_kernel<1, 1, 0, 1, false, 512, 0>": "decode_gemm.o",     # K-class tag 0: K <= 1024
    "decode_gemm_kernel<1, 1, 0, 1, false, 512, 1>": "decode_gemm.down",  # K-class tag 1
    "xstream_gemm_kernel<4, 2, 2, 0, true": "decode_gemm.qkv",   # register-streamed X (round 2)
    "xstream_gemm_kernel<4, 1, 0, 1, false": "decode_gemm.o",
    "xstream_gemm_kernel<19, 1, 0, 1, false": "decode_gemm.down",  # fragment-order activation (act_frag)
    "attn_decode_kernel<64, 7>": "attn_decode",
    "lm_head_kernel<2, 0, false, true": "lm_head_sample",
    "lm_head_kernel<2, 0, false, 1": "lm_head_sample",
    # training kernels (tools/train_kernels.py)
    "logp_entropy_fwd_kernel": "logp_entropy_fwd",
    "logp_bwd_kernel": "logp_bwd",
    "adamw_kernel": "adamw",
    "fa_fwd_kernel": "attn_fwd",
    "fa_dq_kernel": "attn_bwd.dq",
    "fa_dkdv_kernel": "attn_bwd.dkdv",
    "dw_reduce_kernel": "dw_reduce",
    "rmsnorm_bwd_kernel": "rmsnorm_bwd",
    "silu_mul_bwd_kernel": "silu_mul_bwd",
}


def per_kernel(path: str, counter: str) -> dict:
    agg = collections.defaultdict(list)
    with open(path + "/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            key = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("swh::(anonymous namespace)::", ""))
            agg[key].append(float(r["Counter_Value"]))
    return {k: (len(v), sum(v) / len(v)) for k, v in agg.items()}


def main():
    fdir, wdir, out = sys.argv[1:4]
    fetch, write = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
    src = sys.argv[4] if len(sys.argv) > 4 else "tools/bench_decode.py"
    res = {"source": f"rocprofv3 --kernel-trace --pmc FETCH_SIZE | WRITE_SIZE -- python3 {src}",
           "correction": "FETCH_SIZE x2 (gfx950 wide-read tally), KiB -> bytes", "kernels": {}}
    for prefix, name in NAMES.items():
        tf = [k for k in fetch if k.startswith(prefix)]
        tw = [k for k in write if k.startswith(prefix)]
        if tf and tw:
            tmpl = tf[0]
            rd = fetch[tmpl][1] * 2 * 1024
            wr = write[tw[0]][1] * 1024
            res["kernels"][name] = {"template": tmpl, "dispatches": fetch[tmpl][0], "hbm_read_bytes": round(rd),
                                    "hbm_write_bytes": round(wr), "hbm_bytes_per_launch": round(rd + wr)}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
