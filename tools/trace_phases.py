"""Split a rocprofv3 kernel trace of bench.py into GRPO-step phases.

A phase boundary is where the decode kernels start / stop: every run of
decode-engine kernels (decode_gemm / attn_decode / lm_head / embed_gather /
step_advance / sampler) is 'generate', the kernels between two such runs are
'update' (policy forward + backward + optimizer + prefill of the next).
Prints per-window wall span and busy time, and the top kernels of the update
windows.   python tools/trace_phases.py gpurun_out/prof/run_kernel_trace.csv
"""
import collections
import csv
import sys

DEC = ("decode_gemm", "attn_decode", "lm_head", "embed_gather", "step_advance", "lm_sample", "sample_")


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    wins = []
    for r in rows:
        kind = "gen" if any(k in r["Kernel_Name"] for k in DEC) else "upd"
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if wins and wins[-1][0] == kind:
            w = wins[-1]
            w[2] = e
            w[3] += e - s
            w[4].append(r)
        else:
            wins.append([kind, s, e, e - s, [r]])
    # merge tiny windows (a prefill's few kernels) into neighbours for printing
    for k, s, e, busy, rs in wins:
        if len(rs) < 5:
            continue
        print(f"{k} span {(e - s) / 1e6:9.2f} ms busy {busy / 1e6:9.2f} ms kernels {len(rs)}")
    upd = [w for w in wins if w[0] == "upd" and len(w[4]) > 200]
    if upd:
        w = upd[-1]
        c = collections.Counter()
        n = collections.Counter()
        for r in w[4]:
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            c[r["Kernel_Name"][:100]] += d
            n[r["Kernel_Name"][:100]] += 1
        print("last update window top kernels:")
        for k, v in c.most_common(30):
            print(f"  {v / 1e6:8.2f} ms {n[k]:5d}  {k}")


if __name__ == "__main__":
    main(sys.argv[1])
