#!/usr/bin/env python3
"""Summarise a profiles/run_profiles.sh run (rocprofv3 CSVs under gpurun_out/prof) into the
committed evidence under profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary, verbatim
  profiles/<tag>_summary.md         per-kernel time, stream gaps per learn, PMC-derived metrics
  profiles/pmc_traffic.json         HBM bytes per launch per kernel class (bench.py "traffic")

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE and
WRITE_SIZE are KB; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, so it is
doubled; WRITE_SIZE is taken as is.  Counters come from separate --pmc passes (no tracing).

    python tools/prof_summary.py gpurun_out/prof r01 [--config cartpole4096]
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import re
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLASS = {"mb_kernel": "grad", "mbw_kernel": "grad", "grad_kernel": "grad", "eval_kernel": "eval", "gae_kernel": "gae", "gae_pipe_kernel": "gae",
         "pack_kernel": "pack", "slab_reduce_kernel": "slab_reduce",
         "clip_adam_kernel": "clip_adam", "reduce_adam_kernel": "reduce_adam",
         "stats_reduce_kernel": "adv_stats", "fy_build_kernel": "perm",
         "fy_links_kernel": "perm", "fy_solve_kernel": "perm", "shard_count_kernel": "perm",
         "shard_write_kernel": "perm", "next_eval_kernel": "next_eval",
         "gae_aff_kernel": "gae", "fy_walk_scatter_kernel": "perm",
         "fy_walk_mark_kernel": "perm", "gae_stream_probe_kernel": "gae_probe"}


def short(name: str) -> str:
    m = re.search(r"(\w+_kernel)(<[^>]*>)?", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    m = re.search(r"(__amd_\w+)", name)
    return m.group(1) if m else name[:40]


def base(name: str) -> str:
    return short(name).split("<")[0]


def load_pmc(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("tag")
    ap.add_argument("--config", default="cartpole4096")
    ap.add_argument("--gae", type=int, default=0,
                    help="summarise a GAE-only run (gkt, gpmc3, gpmc4 under prof_dir) at this N")
    ap.add_argument("--affine", action="store_true", help="(with --gae) the affine-scan mode")
    a = ap.parse_args()
    P = a.prof_dir
    out_dir = os.path.join(ROOT, "profiles")
    os.makedirs(out_dir, exist_ok=True)
    if a.gae:
        return gae_summary(P, a.tag, a.gae, a.affine, out_dir)
    stats_src = os.path.join(P, "kt", "kt_kernel_stats.csv")
    shutil.copy(stats_src, os.path.join(out_dir, f"{a.tag}_kernel_stats.csv"))
    lines = [f"# {a.tag}: rocprofv3 summary ({a.config})", ""]
    lines += ["Source: `profiles/run_profiles.sh` on one MI355X (gfx950) via gpurun; kernel "
              "durations from `rocprofv3 --kernel-trace --stats`, counters from separate `--pmc` "
              "passes.", ""]
    lines += ["## Kernel time", "", "| kernel | calls | avg µs | min µs | max µs | share |",
              "|---|---|---|---|---|---|"]
    stats = list(csv.DictReader(open(stats_src)))
    for r in stats:
        lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                     f"{float(r['MinNs']) / 1e3:.2f} | {float(r['MaxNs']) / 1e3:.2f} | "
                     f"{float(r['Percentage']):.1f}% |")
    # stream gaps: idle time between consecutive libdppo kernels inside each learn()
    tr = sorted(csv.DictReader(open(os.path.join(P, "kt", "kt_kernel_trace.csv"))),
                key=lambda r: int(r["Start_Timestamp"]))
    learns, cur = [], None
    for r in tr:
        b = base(r["Kernel_Name"])
        if b == "eval_kernel":
            cur = []
            learns.append(cur)
        if cur is not None and b in CLASS:
            cur.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), b))
    rows = []
    for L in learns[1:-1] or learns:
        span = (L[-1][1] - L[0][0]) / 1e3
        busy = sum(e - s for s, e, _ in L) / 1e3
        rows.append((span, busy, len(L)))
    if rows:
        span = sum(r[0] for r in rows) / len(rows)
        busy = sum(r[1] for r in rows) / len(rows)
        nk = rows[0][2]
        lines += ["", "## One learn() on the stream (kernel trace, mean over learns)", "",
                  f"* first-kernel start -> last-kernel end: **{span:.1f} µs**",
                  f"* kernel busy time: {busy:.1f} µs; idle between kernels: {span - busy:.1f} µs "
                  f"over {nk - 1} boundaries ({(span - busy) / max(nk - 1, 1):.2f} µs each)"]
    # PMC-derived
    pmc = {}
    for k in ("pmc1/p1", "pmc2/p2", "pmc3/p3", "pmc4/p4"):
        f = os.path.join(P, k + "_counter_collection.csv")
        if os.path.exists(f):
            for kern, d in load_pmc(f).items():
                pmc.setdefault(kern, {}).update(d)
    traffic = {}
    if pmc:
        lines += ["", "## Counters (per dispatch, mean)", "",
                  "| kernel | MFMA busy | wait any | LDS bank-conflict / LDS active | "
                  "HBM read (2xFETCH) | HBM write | VALU insts | MFMA insts |",
                  "|---|---|---|---|---|---|---|---|"]
        for kern, d in sorted(pmc.items()):
            b = kern.split("<")[0]
            if b not in CLASS:
                continue
            busy = d.get("SQ_BUSY_CYCLES") or 0
            wave = d.get("SQ_WAVE_CYCLES") or 0
            mf = d.get("SQ_VALU_MFMA_BUSY_CYCLES")
            # SQ_BUSY_CYCLES is summed over the 32 shader engines, the MFMA busy cycles over the
            # 1024 SIMDs: per-SIMD busy fraction = mf / 1024 / (busy / 32)
            mfma = f"{mf / busy / 32:.1%}" if mf is not None and busy else "-"
            wait = f"{d['SQ_WAIT_ANY'] / wave:.1%}" if wave and "SQ_WAIT_ANY" in d else "-"
            lds = (f"{d['SQ_LDS_BANK_CONFLICT'] / d['SQ_LDS_IDX_ACTIVE']:.1%}"
                   if d.get("SQ_LDS_IDX_ACTIVE") else "-")
            rd = d.get("FETCH_SIZE")
            wr = d.get("WRITE_SIZE")
            rd_b = 2 * rd * 1024 if rd is not None else None
            wr_b = wr * 1024 if wr is not None else None
            if rd_b is not None and wr_b is not None:
                traffic[CLASS[b]] = int(rd_b + wr_b)
            lines.append(f"| `{kern}` | {mfma} | {wait} | {lds} | "
                         f"{'-' if rd_b is None else f'{rd_b / 1e6:.2f} MB'} | "
                         f"{'-' if wr_b is None else f'{wr_b / 1e6:.2f} MB'} | "
                         f"{d.get('SQ_INSTS_VALU', 0):.0f} | {d.get('SQ_INSTS_MFMA', 0):.0f} |")
        lines += ["", "MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (32 x SQ_BUSY_CYCLES) (1024 SIMDs vs 32 "
                  "shader engines; cross-checked against MFMA instruction count x 32 cycles / "
                  "kernel time); "
                  "wait any = SQ_WAIT_ANY / SQ_WAVE_CYCLES; HBM read = 2 x FETCH_SIZE (gfx950 "
                  "correction), write = WRITE_SIZE."]
        pj = os.path.join(out_dir, "pmc_traffic.json")
        allt = json.load(open(pj)) if os.path.exists(pj) else {}
        allt[a.config] = traffic
        allt["_note"] = ("HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KB x 1024), from "
                         f"profiles/run_profiles.sh via tools/prof_summary.py ({a.tag})")
        json.dump(allt, open(pj, "w"), indent=1, sort_keys=True)
    kt_log = os.path.join(P, "kt.log")
    if os.path.exists(kt_log):
        for ln in open(kt_log):
            if ln.startswith("{"):
                lines += ["", "## bench.py line of the kernel-trace run", "", "```", ln.strip(),
                          "```"]
    # GAE at N = 8192 (bench.py roofline_gae), from the gae_bench.py passes
    gstats = os.path.join(P, "gkt", "gkt_kernel_stats.csv")
    if os.path.exists(gstats):
        shutil.copy(gstats, os.path.join(out_dir, f"{a.tag}_gae8192_kernel_stats.csv"))
        lines += ["", "## GAE at num_envs = 8192 (tools/gae_bench.py, 16 rotating 23 MB sets)", "",
                  "| kernel | calls | avg µs | min µs | max µs |", "|---|---|---|---|---|"]
        for r in csv.DictReader(open(gstats)):
            if base(r["Name"]) in ("gae_pipe_kernel", "gae_kernel"):
                lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | "
                             f"{float(r['AverageNs']) / 1e3:.2f} | {float(r['MinNs']) / 1e3:.2f} | "
                             f"{float(r['MaxNs']) / 1e3:.2f} |")
        g = {}
        for k in ("gpmc3/g3", "gpmc4/g4"):
            f = os.path.join(P, k + "_counter_collection.csv")
            if os.path.exists(f):
                for kern, d in load_pmc(f).items():
                    if base(kern) == "gae_pipe_kernel":
                        g.update(d)
        if "FETCH_SIZE" in g and "WRITE_SIZE" in g:
            rd, wr = 2 * g["FETCH_SIZE"] * 1024, g["WRITE_SIZE"] * 1024
            lines += ["", f"HBM traffic per launch: read {rd / 1e6:.2f} MB (2 x FETCH_SIZE), write "
                      f"{wr / 1e6:.2f} MB (algorithmic: 14 B + 8 B per element = 14.68 + 8.39 MB)"]
            pj = os.path.join(out_dir, "pmc_traffic.json")
            allt = json.load(open(pj)) if os.path.exists(pj) else {}
            allt["gae8192"] = {"gae": int(rd + wr)}
            json.dump(allt, open(pj, "w"), indent=1, sort_keys=True)
        glog = os.path.join(P, "gkt.log")
        if os.path.exists(glog):
            for ln in open(glog):
                if ln.startswith("{"):
                    lines += ["", "```", ln.strip(), "```"]
    open(os.path.join(out_dir, f"{a.tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


def gae_summary(P, tag, N, affine, out_dir):
    """One GAE-only run (tools/gae_bench.py under rocprofv3): kernel stats and HBM traffic per
    launch, keyed gae<N>[_affine] in pmc_traffic.json."""
    key = f"gae{N}" + ("_affine" if affine else "")
    gstats = os.path.join(P, "gkt", "gkt_kernel_stats.csv")
    shutil.copy(gstats, os.path.join(out_dir, f"{tag}_{key}_kernel_stats.csv"))
    lines = [f"# {tag}: GAE at num_envs = {N}" + (" (affine-scan mode)" if affine else ""), "",
             "| kernel | calls | avg µs | min µs | max µs |", "|---|---|---|---|---|"]
    for r in csv.DictReader(open(gstats)):
        if base(r["Name"]).startswith("gae_"):
            lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | "
                         f"{float(r['AverageNs']) / 1e3:.2f} | {float(r['MinNs']) / 1e3:.2f} | "
                         f"{float(r['MaxNs']) / 1e3:.2f} |")
    g = {}
    for k in ("gpmc3/g3", "gpmc4/g4"):
        f = os.path.join(P, k + "_counter_collection.csv")
        if os.path.exists(f):
            for kern, d in load_pmc(f).items():
                if base(kern).startswith("gae_"):
                    g.update(d)
    if "FETCH_SIZE" in g and "WRITE_SIZE" in g:
        rd, wr = 2 * g["FETCH_SIZE"] * 1024, g["WRITE_SIZE"] * 1024
        alg_r, alg_w = 14 * 128 * N, 8 * 128 * N
        lines += ["", f"HBM traffic per launch: read {rd / 1e6:.2f} MB (2 x FETCH_SIZE), write "
                  f"{wr / 1e6:.2f} MB (algorithmic: 14 B + 8 B per element = {alg_r / 1e6:.2f} + "
                  f"{alg_w / 1e6:.2f} MB; ratio {(rd + wr) / (alg_r + alg_w):.3f})"]
        pj = os.path.join(out_dir, "pmc_traffic.json")
        allt = json.load(open(pj)) if os.path.exists(pj) else {}
        allt[key] = {"gae": int(rd + wr)}
        json.dump(allt, open(pj, "w"), indent=1, sort_keys=True)
    glog = os.path.join(P, "gkt.log")
    if os.path.exists(glog):
        for ln in open(glog):
            if ln.startswith("{"):
                lines += ["", "```", ln.strip(), "```"]
    open(os.path.join(out_dir, f"{tag}_{key}_summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
