"""Idle time between consecutive kernels of a rocprofv3 kernel trace, frame by frame (design aid). A bench frame
starts at its k_predict dispatch; for each frame: the span from its first start to the next frame's predict, the sum
of kernel durations, the idle rest, and the largest gaps (graph dispatch + drain between dependent kernels).

    python tools/trace_gaps.py <kernel_trace.csv> [--top 8]
"""
import argparse
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        nm = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", ""))[:40]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), nm))
    rows.sort()
    starts = [i for i, (_, _, n) in enumerate(rows) if n.startswith("k_predict")]
    frames = [rows[starts[i]:starts[i + 1]] for i in range(len(starts) - 1)]
    for fi, fr in enumerate(frames):
        span = fr[-1][1] - fr[0][0]
        busy = sum(e - s for s, e, _ in fr)
        gaps = sorted(((fr[i + 1][0] - fr[i][1], fr[i][2], fr[i + 1][2]) for i in range(len(fr) - 1)), reverse=True)
        pos = [g for g, _, _ in gaps if g > 0]
        print(f"frame {fi}: {len(fr)} kernels, span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, idle "
              f"{(span - busy) / 1e6:.3f} ms ({len(pos)} gaps > 0, mean {sum(pos) / max(1, len(pos)) / 1e3:.2f} us)")
        if fi == len(frames) // 2:
            for g, x, y in gaps[:a.top]:
                print(f"    {g / 1e3:8.2f} us  {x} -> {y}")


if __name__ == "__main__":
    main()
