"""Assemble the committed profile summaries that bench.py reads, from a tools/gpurun/prof_env.sh
run (gpurun_out/prof_<round>) and the shipped build's assembly (make asm -> build/r48_env.s).
Every summary carries source_sha16 (bench.env_source_sha16(): the env kernel sources it was made
from); bench.py ignores a summary whose hash differs from the tree's.

Writes under profiles/<round>/:
  pmc_k_step_n.json      k_step_n (2^20 boards, K = 20 steps per dispatch, the bench's dispatch):
                         SQ counters per dispatch, VALU wave-instructions per board-step
                         (SQ_INSTS_VALU), HBM bytes per dispatch (FETCH_SIZE x 2 + WRITE_SIZE, the
                         gfx950 corrections of /opt/skills/guides/MI355X_MICROARCH.md), and the
                         modelled VALU issue cycles of the shipped loop (tools/isa_hist.py: static
                         instruction mix x measured issue costs, profiles/r02/instr_rate.txt)
  pmc_k_step_2p20.json   k_step (one step per launch, boards through HBM), 2^20 boards
  pmc_k_step_2p26.json   same, 2^26 boards (past the 256 MiB Infinity Cache)
  kernel_stats_bench.csv rocprofv3 --kernel-trace --stats of `python3 bench.py --gpus 1 --steps 20
                         --warmup 5` (the driver's command)
  roofline_from_trace.json  the bench roofline recomputed from that trace (median k_step_n dispatch)
usage: python tools/make_profiles.py <round> [gpurun_out/prof_<round>]"""
import csv
import json
import os
import shutil
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_hist  # noqa: E402
from pmc_summary import summarize  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import env_source_sha16  # noqa: E402

SIMDS, CLOCK_GHZ = 1024, 2.4
BOARDS, K = 1 << 20, 20
KSTEPN = "k_step_nILb1ELb1ELb0ELi1"


def hbm_bytes(pm):
    return (2.0 * pm["FETCH_SIZE"] + pm["WRITE_SIZE"]) * 1024.0


def main():
    rnd = sys.argv[1]
    d = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "prof_" + rnd)
    OUT = os.path.join(ROOT, "profiles", rnd)
    sha = env_source_sha16()
    os.makedirs(OUT, exist_ok=True)
    # ---- k_step_n
    s = summarize("k_step_n", BOARDS // 2, [os.path.join(d, x) for x in ("sqa", "sqb", "stepn_fetch", "stepn_write")])
    pm = s["per_dispatch_mean"]
    bsteps = BOARDS * K
    asm = os.path.join(ROOT, "build", "r48_env.s")
    hist, blocks = isa_hist.analyse(asm, KSTEPN)
    valu = sum(hist.values())
    cyc_opcode = sum(isa_hist.cost(k) * v for k, v in hist.items())
    mdl = isa_hist.model(isa_hist.loop_lines(asm, KSTEPN)[0])
    cyc = mdl["modelled_cycles"]      # opcode costs + literal / inline-constant costs, SGPR-read bound
    s.update({
        "kernel": "k_step_n<RANDOM=1,AUTO_RESET=1,REWARD=0,NP=1>",
        "boards": BOARDS, "steps_per_dispatch": K, "board_steps_per_dispatch": bsteps,
        "source": "rocprofv3 --pmc passes (one counter group each) of tools/prof_stepn.py 20 300, tools/gpurun/prof_env.sh",
        "source_sha16": sha,
        "valu_wave_instr_per_board_step": pm["SQ_INSTS_VALU"] / bsteps,
        "hbm_bytes_per_dispatch": hbm_bytes(pm),
        "algorithmic_bytes_per_dispatch": 34 * BOARDS,
        "isa_loop": {"asm": "build/r48_env.s (make asm)", "blocks": blocks, "valu_per_wave_pass": valu,
                     "board_steps_per_wave_pass": 128, "modelled_issue_cycles_per_wave_pass": cyc,
                     "opcode_only_cycles_per_wave_pass": cyc_opcode, "operand_model": mdl,
                     "histogram": dict(hist.most_common())},
        "modelled_cycles_per_board_step": cyc / 128.0,
        "opcode_only_cycles_per_board_step": cyc_opcode / 128.0,
        "counter_valu_frac": pm["SQ_INSTS_VALU"] / (s["pmc_dispatch_ns_mean"] * 1e-9) / 1e9 / (SIMDS * CLOCK_GHZ / 2.0),
        "note": "a wave pass = one step of the 128 boards of a wave (64 lanes x a board pair); issue costs per "
                "instruction from profiles/r02/instr_rate.txt (8 independent chains x 8 waves per SIMD), plus the "
                "round-5 operand costs (profiles/r05/env/instr_rate_r05.txt: literal +0.26, inline constant +0.16 "
                "cycles on full-rate instructions; SGPR-reading VALU limited to one per 4.2 cycles per SIMD, a "
                "separate bound). counter_valu_frac = SQ_INSTS_VALU / profiled dispatch time / (1024 SIMDs x 2.4 GHz "
                "/ 2): the counter-only fraction, no cost model",
    })
    json.dump(s, open(os.path.join(OUT, "pmc_k_step_n.json"), "w"), indent=1)
    # ---- k_step at 2^20 and 2^26
    for tag, n in (("2p20", 1 << 20), ("2p26", 1 << 26)):
        k = summarize("k_step<", n // 2, [os.path.join(d, "k%s_fetch" % tag[2:]), os.path.join(d, "k%s_write" % tag[2:])])
        pk = k["per_dispatch_mean"]
        k.update({"kernel": "k_step<RANDOM=1,AUTO_RESET=1,REWARD=0>", "boards": n,
                  "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of tools/prof_kstep.py, tools/gpurun/prof_env.sh",
                  "source_sha16": sha,
                  "hbm_bytes_per_launch": hbm_bytes(pk), "algorithmic_bytes_per_launch": 34 * n,
                  "traffic_over_algorithmic": hbm_bytes(pk) / (34.0 * n),
                  "correction": "bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (KiB; gfx950 FETCH_SIZE halving)"})
        if n <= (1 << 22):
            k["cache_note"] = ("36 MB per step fits the 256 MiB Infinity Cache: these fabric-side counters include "
                               "MALL hits, so this is traffic past L2, not HBM traffic")
        json.dump(k, open(os.path.join(OUT, "pmc_k_step_%s.json" % tag), "w"), indent=1)
    # ---- kernel trace of the driver's bench command
    shutil.copy(os.path.join(d, "kt", "kt_kernel_stats.csv"), os.path.join(OUT, "kernel_stats_bench.csv"))
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            for r in csv.DictReader(open(os.path.join(d, "kt", "kt_kernel_trace.csv")))
            if "k_step_n" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == BOARDS // 2]
    med = statistics.median(durs)
    cyc_bs = cyc / 128.0
    ach = cyc_bs * bsteps / (med * 1e-9) / 1e9
    rt = {"kernel": "k_step_n<RANDOM=1,AUTO_RESET=1,REWARD=0,NP=1>", "source_sha16": sha, "dispatches": len(durs),
          "median_dispatch_ns": med, "mean_dispatch_ns": sum(durs) / len(durs),
          "board_steps_per_dispatch": bsteps,
          "modelled_issue_cycles_per_board_step": cyc_bs,
          "opcode_only_cycles_per_board_step": cyc_opcode / 128.0,
          "frac_opcode_only": cyc_opcode / 128.0 * bsteps / (med * 1e-9) / 1e9 / (SIMDS * CLOCK_GHZ),
          "achieved_G_issue_cycles_per_s": ach, "peak_G_issue_cycles_per_s": SIMDS * CLOCK_GHZ,
          "frac": ach / (SIMDS * CLOCK_GHZ),
          "valu_wave_instr_per_board_step_pmc": pm["SQ_INSTS_VALU"] / bsteps,
          "instr_rate_frac": pm["SQ_INSTS_VALU"] / (med * 1e-9) / 1e9 / (SIMDS * CLOCK_GHZ / 2.0),
          "formula": "frac = modelled issue cycles per board-step (opcode + operand costs, isa_hist.model) x 2^20 x 20 / "
                     "median dispatch time / (1024 SIMDs x 2.4 GHz); instr_rate_frac = SQ_INSTS_VALU per dispatch / median dispatch time / "
                     "(1024 SIMDs x 2.4 GHz / 2 cycles per full-rate wave64 instruction)",
          "trace": "profiles/%s/kernel_stats_bench.csv (rocprofv3 --kernel-trace --stats of python3 bench.py --gpus 1 "
                   "--steps 20 --warmup 5)" % rnd}
    json.dump(rt, open(os.path.join(OUT, "roofline_from_trace.json"), "w"), indent=1)
    print(json.dumps(rt, indent=1))


if __name__ == "__main__":
    main()
