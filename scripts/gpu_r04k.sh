#!/bin/bash
# lookup A/B, then C5's counters refreshed for the renumbered view's launch shape
set -o pipefail
bash scripts/gpu_shim_ab.sh r04k 4 || exit 1
bash scripts/gpu_roofline.sh r04k_c5 C5 1.0 'k_relax\(|k_relax_wl\(|k_relax_wlp\(' || exit 1
