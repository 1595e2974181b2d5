#!/usr/bin/env python3
"""Per-frame kernel-time budget by phase from a rocprofv3 --kernel-trace CSV.

    python tools/frame_budget.py <kernel_trace.csv> [--md out.md]

Under --kernel-trace the graph's streams run one after another, so the sums are SERIAL kernel time
per frame (frames = patchify launches); the replayed frame overlaps the side encoders and the
decoder chains, so it is shorter.  FLOP per phase: the algorithmic work (SURVEY 8d shapes); fraction
of the 2.5 PFLOP/s dense bf16 / f16 MFMA peak; "to 15.4 ms" = the time the phase would take at 0.5
of peak (the north-star's 50 % roofline, 19.247 TFLOP at 65 frames/s)."""
import argparse
import csv
import re
from collections import defaultdict

PEAK = 2.5e15
GF = 1e9
# per-frame algorithmic FLOP of the ViT phases (M = 20195 patch rows, 577 x 2 side rows, 24 blocks)
PATCH = {"qkv": 24 * 2 * 20195 * 3072 * 1024, "proj + fc2": 24 * 2 * 20195 * 1024 * (1024 + 4096),
         "fc1": 24 * 2 * 20195 * 4096 * 1024, "attention (patch)": 24 * 35 * 16 * 4 * 577 * 577 * 64}
SIDE = 24 * 2 * (2 * 577 * 1024 * (3072 + 1024 + 4096 + 4096) + 16 * 4 * 577 * 577 * 64)
TOTAL = 19.247e12


def classify(name, wgs):
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    if "gemm_8ph320_kernel" in n and ", 0, 2>" in n:
        return "qkv"
    if "gemm_p8ph_kernel" in n and "false, 0, false, false, true>" in n:   # (round 5: qkv on the persistent engine)
        return "qkv"
    if "gemm_8ph320_kernel" in n and ", 16, 3>" in n or "gemm_8ph320_kernel" in n and ", 16, 1>" in n:
        return "proj + fc2"
    if "gemm_p8ph_kernel" in n and "true>" in n and ", 2," in n:
        return "fc1"
    if "ln_merge_kernel" in n or "ln_stats_kernel" in n:
        return "LN (patch: stats, merge)"
    if "attn_kernel" in n:
        return "attention (patch)" if wgs > 1000 else "side encoders"
    if "gemm_big_kernel" in n and "true, false>" in n and "128, 128" in n:
        return "side encoders"
    if "ln_kernel<KBF16" in n:
        return "side encoders"
    if "gemm_cv3_kernel" in n and ", 12>" in n:       # (12-row tiles: the 384^2 / 192^2 convs)
        return "decoder / encoder maps (other GEMMs)"
    if "gemm_cv3_kernel" in n or ("gemm_big_kernel" in n and ("512, 128" in n)):
        return "decoder 768^2 convs + head"
    if "gemm_p8ph_kernel" in n or "gemm_sk_kernel" in n or "gemm_big_kernel" in n or "gemm_kernel" in n \
            or "gemm_pbig" in n:
        return "decoder / encoder maps (other GEMMs)"
    if n.startswith("void at::") or "rocclr" in n or "rocblas" in n or "Cijk" in n:
        return "torch / copies (outside the engine)"
    return "small kernels (patchify, merge, LN, epilogues)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--md")
    ap.add_argument("--alone-md", help="per-kernel alone times (average over the serial frames) as markdown")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args()
    # frames = runs of launches from one patchify launch to the next; only frames whose launches never
    # overlap (a serial frame: the trace serialised that replay, or an eager serial forward) are summed,
    # so a launch's duration is its own time alone on the chip, not time spent waiting for CUs
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                   int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))) for r in csv.DictReader(open(a.trace)))
    groups, cur = [], None
    for r in rows:
        if "patchify_kernel" in r[2]:
            cur = []
            groups.append(cur)
        if cur is not None:
            cur.append(r)
    tot = defaultdict(float)
    per = defaultdict(lambda: [0, 0.0])       # (kernel, workgroups) -> [launches, us] over the serial frames
    frames = skipped = 0
    spans = sorted(max(r[1] for r in g) - g[0][0] for g in groups)
    med = spans[len(spans) // 2]
    for g in groups:
        if max(r[1] for r in g) - g[0][0] > 1.5 * med:   # a cold first forward (code-object loads)
            skipped += 1
            continue
        # overlapped time (ns) of the frame's launches; a frame counts as serial below 1 % of its span
        # (the serial eager frame can have a launch starting a few us before the previous one retires)
        end, olap = 0, 0
        for t0, t1, _, _ in g:
            if t0 < end:
                olap += min(end, t1) - t0
            end = max(end, t1)
        if olap > 0.01 * (end - g[0][0]):
            skipped += 1
            continue
        if a.verbose:
            fc1 = [(t1 - t0) / 1e3 for t0, t1, n, w in g if classify(n, w) == "fc1"]
            print(f"serial frame at {g[0][0]}: span {(end - g[0][0]) / 1e6:.3f} ms, overlap {olap / 1e3:.1f} us, "
                  f"fc1 avg {sum(fc1) / max(len(fc1), 1):.1f} us")
        frames += 1
        for t0, t1, name, wgs in g:
            tot[classify(name, wgs)] += (t1 - t0) * 1e-3
            k = per[(re.sub(r"\(anonymous namespace\)::", "", name).split("(")[0], wgs)]
            k[0] += 1
            k[1] += (t1 - t0) * 1e-3
    if frames == 0:
        raise SystemExit("no serial frame in the trace (every frame's launches overlap)")
    flop = dict(PATCH)
    flop["side encoders"] = SIDE
    rest = TOTAL - sum(flop.values())
    lines = [f"serial frames in the trace: {frames} (skipped {skipped}: launches overlapping > 1 %, or a cold first forward); kernel time per "
             f"frame by phase", "",
             "| phase | ms / frame | GFLOP / frame | TFLOP/s | fraction of peak | ms at 0.5 of peak | ms to lose |",
             "|---|---:|---:|---:|---:|---:|---:|"]
    order = ["qkv", "attention (patch)", "proj + fc2", "fc1", "LN (patch: stats, merge)", "side encoders",
             "decoder / encoder maps (other GEMMs)", "decoder 768^2 convs + head",
             "small kernels (patchify, merge, LN, epilogues)", "torch / copies (outside the engine)"]
    tsum = 0.0
    for k in order:
        ms = tot.get(k, 0.0) / frames / 1e3
        if not k.startswith("torch"):          # (set-up kernels of the profiled run: weight packing etc.)
            tsum += ms
        f = flop.get(k)
        if f and ms > 0:
            tf = f / (ms * 1e-3) / 1e12
            half = f / (0.5 * PEAK) * 1e3
            lines.append(f"| {k} | {ms:.3f} | {f / GF:.0f} | {tf:.0f} | {tf * 1e12 / PEAK:.3f} | {half:.3f} | "
                         f"{max(ms - half, 0):.3f} |")
        else:
            lines.append(f"| {k} | {ms:.3f} | | | | | |")
    dec = tot.get("decoder / encoder maps (other GEMMs)", 0) + tot.get("decoder 768^2 convs + head", 0)
    dms = dec / frames / 1e3
    lines.append(f"| (decoder + heads + encoder maps together) | {dms:.3f} | {rest / GF:.0f} | "
                 f"{rest / (dms * 1e-3) / 1e12:.0f} | {rest / (dms * 1e-3) / PEAK:.3f} | {rest / (0.5 * PEAK) * 1e3:.3f} | "
                 f"{max(dms - rest / (0.5 * PEAK) * 1e3, 0):.3f} |")
    lines.append(f"| **serial sum (engine kernels)** | **{tsum:.3f}** | {TOTAL / GF:.0f} | | | {TOTAL / (0.5 * PEAK) * 1e3:.3f} | |")
    out = "\n".join(lines)
    print(out)
    if a.md:
        open(a.md, "w").write(out + "\n")
    if a.alone_md:
        al = [f"Per-kernel ALONE times: the {frames} serial frames of `{a.trace.split('/')[-1]}` (every launch on one "
              f"stream, so each ran alone on the chip); kernel, workgroups, launches per frame, average us per launch, "
              f"us per frame", "", "| kernel | workgroups | launches / frame | avg us | us / frame | phase |",
              "|---|---:|---:|---:|---:|---|"]
        for (name, wgs), (n, us) in sorted(per.items(), key=lambda kv: -kv[1][1]):
            if us / frames < 5.0:
                continue
            al.append(f"| `{name[:90]}` | {wgs} | {n / frames:g} | {us / n:.2f} | {us / frames:.1f} | "
                      f"{classify(name, wgs)} |")
        open(a.alone_md, "w").write("\n".join(al) + "\n")


if __name__ == "__main__":
    main()
