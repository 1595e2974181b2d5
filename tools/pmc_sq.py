#!/usr/bin/env python3
"""Per-kernel MFMA utilisation and wave-state split of one eager forward from rocprofv3 --pmc passes.

    python tools/pmc_sq.py <pass1 counter_collection.csv> [<pass2 counter_collection.csv>] [--json out.json]

Pass 1 (tools/gpu_check.sh ... sq): SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA + GRBM_GUI_ACTIVE.
Pass 2 (optional): SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU + GRBM_GUI_ACTIVE.

Definitions (MI355X_MICROARCH.md, rocprofv3 PMC slots and DVFS give-back):
  active cycles per XCD  A = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs)
  MFMA util              = SQ_VALU_MFMA_BUSY_CYCLES / (A * 1024 SIMDs)    (busy cycles summed over SIMDs)
  wave-state split       = SQ_WAIT_ANY (parked on s_waitcnt / barrier), SQ_WAIT_INST_ANY (issue-stalled),
                           SQ_ACTIVE_INST_ANY (issuing), as fractions of SQ_WAVE_CYCLES (disjoint, ~sum to 1)
  effective clock        = A / duration is not available here (no timing in a PMC pass); the kernel-trace
                           durations come from the --stats run of the same command.
The last forward (from the last patchify dispatch) is used; rows grouped by (kernel, grid).
"""
import argparse
import csv
import json
import re
from collections import defaultdict


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\(.*$", "", n).replace("void ", "")
    return n[:72]


def load(path):
    """{dispatch_id: (kernel, workgroups, {counter: value})} of the last forward."""
    d = {}
    for r in csv.DictReader(open(path)):
        i = int(r["Dispatch_Id"])
        if i not in d:
            wg = int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"]))
            d[i] = (r["Kernel_Name"], wg, {})
        d[i][2][r["Counter_Name"]] = d[i][2].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(d)
    starts = [i for i in ids if "patchify_kernel" in d[i][0]]
    if starts:
        ids = [i for i in ids if i >= starts[-1]]
    return [d[i] for i in ids]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pass1")
    ap.add_argument("pass2", nargs="?")
    ap.add_argument("--json")
    args = ap.parse_args()
    rows = load(args.pass1)
    rows2 = load(args.pass2) if args.pass2 else None
    if rows2 is not None:
        assert len(rows2) == len(rows), (len(rows), len(rows2))
        for (n1, _, c1), (n2, _, c2) in zip(rows, rows2):
            assert n1 == n2
            for k, v in c2.items():
                c1.setdefault(k, v)
    g = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(int)
    for name, wg, c in rows:
        k = (short(name), wg)
        calls[k] += 1
        for cn, v in c.items():
            g[k][cn] += v
    tot_active = sum(v.get("GRBM_GUI_ACTIVE", 0.0) for v in g.values())
    print(f"one eager forward: {len(rows)} dispatches\n")
    cols = "| kernel | WGs | calls | share of active | MFMA util | wait | stall | issue |"
    extra = rows2 is not None
    if extra:
        cols += " VALU/MFMA | LDS/MFMA | LDS bank confl. |"
    print(cols)
    print("|---|---:|---:|---:|---:|---:|---:|---:|" + ("---:|---:|---:|" if extra else ""))
    out = []
    for k, c in sorted(g.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0.0)):
        A = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        wc = max(c.get("SQ_WAVE_CYCLES", 0.0), 1.0)
        util = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (A * 1024.0) if A else 0.0
        rec = {"kernel": k[0], "workgroups": k[1], "calls": calls[k],
               "active_share": c.get("GRBM_GUI_ACTIVE", 0.0) / tot_active if tot_active else 0.0,
               "mfma_util": util, "wait": c.get("SQ_WAIT_ANY", 0.0) / wc,
               "stall": c.get("SQ_WAIT_INST_ANY", 0.0) / wc, "issue": c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc,
               "counters": dict(c)}
        line = (f"| `{k[0]}` | {k[1]} | {calls[k]} | {rec['active_share']:.3f} | {util:.3f} | {rec['wait']:.2f} | "
                f"{rec['stall']:.2f} | {rec['issue']:.2f} |")
        if extra:
            m = max(c.get("SQ_INSTS_MFMA", 0.0), 1.0)
            rec["valu_per_mfma"] = c.get("SQ_INSTS_VALU", 0.0) / m
            rec["lds_per_mfma"] = c.get("SQ_INSTS_LDS", 0.0) / m
            rec["lds_bank_conflict_frac"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(c.get("SQ_LDS_IDX_ACTIVE", 0.0), 1.0)
            line += f" {rec['valu_per_mfma']:.2f} | {rec['lds_per_mfma']:.2f} | {rec['lds_bank_conflict_frac']:.3f} |"
        print(line)
        out.append(rec)
    if args.json:
        json.dump({"kernels": out}, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
