"""Timeline of one batched TPKE step from a rocprofv3 --kernel-trace CSV: every dispatch from shortly before the N-th
launch of k_tpke_ct_prepare_h at the bench size (>= 47,000 lanes) to the next one, with start / end / duration in ms
relative to that launch, and the queue / stream it ran on (what overlaps what, and what waits).
Usage: python tools/step_timeline.py <run_kernel_trace.csv> N
"""
import csv
import sys


def main(path, which):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows)
           if r["Kernel_Name"].startswith("k_tpke_ct_prepare_h") and int(r["Grid_Size_X"]) >= 47000]
    i0, i1 = idx[which], idx[which + 1]
    t0, t1 = int(rows[i0]["Start_Timestamp"]), int(rows[i1]["Start_Timestamp"])
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < t0 - 2_000_000 or s >= t1:
            continue
        print(f"{(s - t0) / 1e6:8.2f} {(e - t0) / 1e6:8.2f} {(e - s) / 1e6:7.2f} q{r['Queue_Id']:>3s} "
              f"s{r['Stream_Id']:>3s} {r['Kernel_Name'][:34]:34s} {r['Grid_Size_X']}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
