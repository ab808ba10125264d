"""Concurrency of two streams in a rocprofv3 kernel trace (tuning aid, not part of
the product): for the last `window_ms` of the trace, each stream's busy time
(union of its kernels' [start, end)) and the time both streams had a kernel
running, plus the mean kernel duration per stream.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/dual_decode.py --iters 1
    python tools/stream_overlap.py OUT/.../run_kernel_trace.csv [window_ms]
"""
import csv
import sys


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def inter(a, b):
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main(path, window_ms=20.0):
    rows = list(csv.DictReader(open(path)))
    key = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r[key]) for r in rows]
    t_end = max(e for _, e, _ in ks)
    t0 = t_end - int(window_ms * 1e6)
    ks = [k for k in ks if k[0] >= t0]
    streams = {}
    for s, e, q in ks:
        streams.setdefault(q, []).append((s, e))
    top = sorted(streams.items(), key=lambda kv: -sum(e - s for s, e in kv[1]))[:2]
    span = max(e for _, e, _ in ks) - min(s for s, _, _ in ks)
    us = [union(v) for _, v in top]
    for (q, v), u in zip(top, us):
        busy = sum(e - s for s, e in u)
        print(f"stream {q}: {len(v)} kernels, busy {busy / 1e3:.1f} us of {span / 1e3:.1f} us "
              f"({100 * busy / span:.0f} %), mean kernel {sum(e - s for s, e in v) / len(v) / 1e3:.2f} us")
    if len(us) == 2:
        both = inter(us[0], us[1])
        print(f"both streams busy {both / 1e3:.1f} us ({100 * both / span:.0f} % of the span)")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 20.0)
