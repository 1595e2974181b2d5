#!/usr/bin/env python3
"""fc1 on the persistent engine with and without its GELU epilogue, back to back, for a rocprofv3
PMC pass (GRBM_GUI_ACTIVE + kernel trace): the clock the chip holds under each variant
(MI355X_MICROARCH.md, DVFS give-back: effective clock = GRBM_GUI_ACTIVE / 8 / kernel wall time).

    rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d out -o pmc --output-format csv -- \
        python3 tools/gelu_clock.py
    python3 tools/gelu_clock.py --report out/pmc_counter_collection.csv out/pmc_kernel_trace.csv
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run():
    import torch

    sys.path.insert(0, os.path.join(ROOT, "ml-depth-pro-video_amd"))
    from depth_pro import ops  # noqa: E402
    from depth_pro._lib import DP_ACT_GELU, DP_TILE_P8PH_256x256  # noqa: E402

    dev = torch.device("cuda:0")
    dt = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    M, N, K = 20195, 4096, 1024
    A = torch.randn(M, K, device=dev, generator=g).to(dt)
    B = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(dt)
    bias = torch.randn(N, device=dev, generator=g)
    colsum = B.float().sum(1).contiguous()
    rs = torch.rand((M + 1) // 2 * 2 + 256, 2, device=dev, generator=g) + 0.5
    C = torch.empty(M, N, device=dev, dtype=dt)
    ws = ops.gemm_workspace(dev)
    for act in (DP_ACT_GELU, 0, DP_ACT_GELU, 0):
        for _ in range(40):
            ops.gemm(A, B, C, M=M, N=N, K=K, bias=bias, act=act, ln_in=(None, colsum), ln_rs_in=rs,
                     tile=DP_TILE_P8PH_256x256, workspace=ws)
        torch.cuda.synchronize()


def report(pmc_csv, trace_csv):
    import csv
    import statistics

    trace = {r["Dispatch_Id"]: r for r in csv.DictReader(open(trace_csv)) if "p8ph" in r["Kernel_Name"]}
    grbm = {}
    for r in csv.DictReader(open(pmc_csv)):
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and r["Dispatch_Id"] in trace:
            grbm[r["Dispatch_Id"]] = grbm.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    rows = {}
    for d, r in trace.items():
        if d not in grbm:
            continue
        act = "GELU" if ", 2, " in r["Kernel_Name"] else "none"
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        rows.setdefault(act, []).append((us, grbm[d] / 8 / us / 1e3))
    for act, v in rows.items():
        print(f"fc1 act={act:4s}: {len(v)} launches, median {statistics.median(x for x, _ in v):6.1f} us, "
              f"effective clock median {statistics.median(c for _, c in v):.3f} GHz")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--report":
        report(sys.argv[2], sys.argv[3])
    else:
        run()
