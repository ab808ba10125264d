"""Where the training half-step's time goes, stream by stream, from a
rocprofv3 kernel trace of tools/train_kernels.py (tuning aid, not part of
the product).

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/train_kernels.py --reps 1
    python tools/critical_path.py OUT/.../run_kernel_trace.csv

The last `window` ms of the trace (the timed step; without --whole, from the
last host gap > 5 ms on) is analysed: per stream
its busy time and idle gaps; for the busiest stream (the compute stream) each
gap is attributed to what the other streams ran meanwhile (the fence on the
weight-gradient GEMMs, dK/dV, ...), and the kernels are grouped by family with
their summed durations.
"""
import collections
import csv
import re
import sys


def family(name: str) -> str:
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = re.sub(r"^void ", "", n).split("(")[0]
    if n.startswith(("Cijk", "Custom_Cijk")):
        m = re.search(r"MT(\d+x\d+x\d+)", n)
        return "GEMM " + (m.group(1) if m else "")
    n = re.sub(r"^swh::", "", n)
    n = re.sub(r"^at::native::", "aten::", n)
    return n[:60]


def main(path: str, window_ms: float = 200.0, cut_gaps: bool = True):
    rows = list(csv.DictReader(open(path)))
    key = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r[key], r["Kernel_Name"]) for r in rows]
    ks.sort()
    t_end = max(e for _, e, _, _ in ks)
    # the timed step: everything after the last gap > 5 ms (host sync between reps), capped at the window
    starts = [s for s, _, _, _ in ks]
    cut = ks[0][0]
    prev_end = ks[0][1]
    for s, e, _, _ in ks:
        if cut_gaps and s - prev_end > 5e6:
            cut = s
        prev_end = max(prev_end, e)
    cut = max(cut, t_end - int(window_ms * 1e6))
    ks = [k for k in ks if k[0] >= cut]
    t0 = ks[0][0]
    span = max(e for _, e, _, _ in ks) - t0
    by = collections.defaultdict(list)
    for k in ks:
        by[k[2]].append(k)
    print(f"window {span / 1e6:.2f} ms, {len(ks)} kernels, streams {sorted(by)}")
    iv = sorted((b, e) for b, e, _, _ in ks)  # GPU idle = no stream running anything
    busy, (cs, ce), idle = 0, iv[0], []
    for b, e in iv[1:]:
        if b > ce:
            busy += ce - cs
            idle.append((b - ce, (ce - t0) / 1e6))
            cs, ce = b, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    small = sum(g for g, _ in idle if g < 50e3)
    print(f"GPU busy (any stream) {busy / 1e6:.2f} ms, idle {(span - busy) / 1e6:.2f} ms "
          f"({small / 1e6:.2f} ms in gaps < 50 us); largest idle gaps (ms at ms): "
          + ", ".join(f"{g / 1e6:.2f}@{t:.1f}" for g, t in sorted(idle, reverse=True)[:10]))
    main_s = max(by, key=lambda s: sum(e - b for b, e, _, _ in by[s]))
    for s, lst in sorted(by.items()):
        busy = sum(e - b for b, e, _, _ in lst)
        print(f"stream {s:>4}: {len(lst):5d} kernels, busy {busy / 1e6:8.2f} ms" + ("  <- compute" if s == main_s else ""))
    # gaps of the compute stream and what ran elsewhere meanwhile
    lst = by[main_s]
    gap_total = 0
    blame = collections.Counter()
    for (b0, e0, _, n0), (b1, _, _, n1) in zip(lst, lst[1:]):
        g = b1 - e0
        if g <= 2000:  # under 2 us: launch boundary
            continue
        gap_total += g
        over = collections.Counter()
        for b, e, s, n in ks:
            if s != main_s and b < b1 and e > e0:
                over[family(n)] += min(e, b1) - max(b, e0)
        who = over.most_common(1)[0][0] if over else "(nothing: host / boundary)"
        blame[f"before {family(n1)} | elsewhere: {who}"] += g
    big = sorted(((b1 - e0, e0 - t0, n0, n1) for (b0, e0, _, n0), (b1, _, _, n1) in zip(lst, lst[1:])), reverse=True)
    print("\nlargest single compute-stream gaps (ms, at ms, after -> before):")
    for g, at, n0, n1 in big[:12]:
        print(f"  {g / 1e6:7.3f} at {at / 1e6:7.2f}  {family(n0)} -> {family(n1)}")
    print(f"\ncompute-stream gaps > 2 us: {gap_total / 1e6:.2f} ms")
    for k, v in blame.most_common(15):
        print(f"  {v / 1e6:7.2f} ms  {k}")
    fam = collections.Counter()
    cnt = collections.Counter()
    for b, e, s, n in ks:
        fam[(s == main_s, family(n))] += e - b
        cnt[(s == main_s, family(n))] += 1
    print("\nkernel families (C = compute stream, S = other streams):")
    for (m, f), v in fam.most_common(30):
        print(f"  {'C' if m else 'S'} {v / 1e6:7.2f} ms  {cnt[(m, f)]:5d}  {f}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 200.0, "--whole" not in sys.argv)
