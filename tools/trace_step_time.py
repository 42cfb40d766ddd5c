#!/usr/bin/env python3
"""Per-step device time of the env step from a rocprofv3 --kernel-trace CSV.

r48_env_step_n runs 2^20 boards as two shard chains whose k_step dispatches (n/2 boards each)
overlap, so rocprofv3's per-dispatch average is not the per-step time. This tool takes the
timed region's graph-replayed k_step dispatches (grid = n/2 lanes), merges overlapping
intervals, and divides the busy time by the number of steps (dispatches / chains). The result
is what bench.py's roofline.step_ms_device_events_timed_region measures with HIP events.

    python tools/trace_step_time.py gpurun_out/prof/run_kernel_trace.csv --boards 1048576
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--boards", type=int, default=1 << 20)
    ap.add_argument("--chains", type=int, default=2)
    ap.add_argument("--skip", type=int, default=0, help="leading k_step dispatches to drop (warm-up)")
    a = ap.parse_args()
    lanes = a.boards // a.chains
    iv = []
    with open(a.trace) as f:
        for row in csv.DictReader(f):
            # one board pair per lane: a launch over `lanes` boards has lanes / 2 threads
            if "k_step<" in row["Kernel_Name"] and int(row["Grid_Size_X"]) * 2 == lanes:
                iv.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    iv.sort()
    iv = iv[a.skip:]
    busy, cur_s, cur_e, dur = 0, None, None, []
    for s, e in iv:
        dur.append(e - s)
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    steps = len(iv) / a.chains
    step_us = busy / steps / 1e3
    print("k_step dispatches of %d boards: %d (= %.0f steps x %d chains)" % (lanes, len(iv), steps, a.chains))
    print("avg dispatch duration: %.3f us" % (sum(dur) / len(dur) / 1e3))
    print("busy time (union of overlapping dispatches) per step: %.3f us" % step_us)
    print("=> %.1f G env-steps/s, %.0f GB/s algorithmic (34 B/board-step)"
          % (a.boards / step_us / 1e3, a.boards * 34 / step_us / 1e3))


if __name__ == "__main__":
    main()
