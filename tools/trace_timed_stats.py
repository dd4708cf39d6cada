"""Per-kernel duration summary of the TIMED launches only, from a rocprofv3
kernel trace of `python3 bench.py --gpus 1 --steps K --warmup W`.

rocprofv3 --stats averages every launch of the run, the W untimed warmup steps
included (the first ones run at a lower clock); the bench line's roofline is
measured over the K timed steps.  This keeps each kernel's last K x B launches
(B launches per step) so the two can be compared launch for launch.

  python tools/trace_timed_stats.py TRACE.csv K B OUT.csv
"""
import collections
import csv
import sys


def main():
    trace, k, b, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    by = collections.defaultdict(list)
    for r in rows:
        by[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Note"])
        for name, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            if len(d) >= k * b:
                d = d[-k * b:]
                note = f"last {k}x{b} launches (the timed steps)"
            else:
                note = "all launches"
            w.writerow([name, len(d), sum(d), sum(d) / len(d), min(d), max(d), note])


if __name__ == "__main__":
    main()
