#!/bin/bash
# round 5, run y: the split draw's pool (per-worker futex wake) — thread scaling + per-thread times
set -o pipefail
O=gpurun_out/r05/y
mkdir -p $O
timeout -k 10 200 python -u scripts/diag/diag_cpu_mask_threads.py > $O/mask_threads.json 2> $O/mask_threads.err && \
HGD_RNG_DEBUG=1 timeout -k 10 100 python - 2> $O/debug.txt <<'PY'
import ctypes, torch
from hypergraph_diffusion_for_recommendation_amd import _native as nat
lib = nat.load()
n = 3 * 2473226
mask = torch.empty(n, dtype=torch.uint8, pin_memory=True)
mask.fill_(0)
kept = ctypes.c_int64()
for th in (2, 16):
    for rep in range(4):
        st = torch.get_rng_state()
        nat.check(lib.hgd_torch_cpu_keep_mask_threads(st.data_ptr(), st.numel(), n, 0.5,
                                                      mask.data_ptr(), ctypes.byref(kept), th), "x")
PY
