#!/bin/bash
# Frame-time ablations (GPU box): each run drops one stage of the forward (outputs invalid).
cd "$GRAFT_REPO_ROOT"
for A in "" side attn ln vitgemm decoder head "side,attn,ln,vitgemm"; do
  v=$(DP_ABLATE=$A timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')
  echo "ablate=[$A] $v"
done
