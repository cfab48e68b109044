#!/bin/bash
# Push vs pull relax traffic (verdict r03 item 1), C4 and C5
set -o pipefail
TAG=${1:?tag}
O=gpurun_out/$TAG
PULL='k_relax\(|k_relax_wl\(|k_relax_wlp\(|k_compact'
PUSH='k_push|k_pred_pass|k_fold|k_compact'
for cfg in C4 C5; do
  bash _exp/scripts/ab_counters.sh $O/${cfg}_pull $cfg "--csr-variant 1" "$PULL" || exit 1
  bash _exp/scripts/ab_counters.sh $O/${cfg}_push $cfg "--csr-variant 2" "$PUSH" || exit 1
done
