#!/bin/bash
# round 6 (q): the side encoders' frame cost on the final tree, four alternating samples on one box
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06q; mkdir -p $O
for R in 1 2 3 4; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/side_$R.json 2> $O/side_$R.err
  DP_ABLATE=side timeout -k 10 300 python -u bench.py --ab --no-cpu-baseline --steps 40 > $O/noside_$R.json 2> $O/noside_$R.err
done
python3 - <<'PY' > $O/side.txt
import json
rows = []
for r in range(1, 5):
    a = json.load(open(f"gpurun_out/r06q/side_{r}.json")); b = json.load(open(f"gpurun_out/r06q/noside_{r}.json"))
    rows.append((a["ms_per_step"], b["ms_per_step"]))
    print(f"sample {r}: full {a['ms_per_step']:.3f} ms ({a['value']} fps), side ablated {b['ms_per_step']:.3f} ms -> side {a['ms_per_step'] - b['ms_per_step']:.3f} ms")
print(f"mean side cost {sum(x - y for x, y in rows) / len(rows):.3f} ms")
PY
