set -o pipefail
O=gpurun_out/r04d
bash scripts/ab_counters.sh $O/C4_pull C4 "--csr-variant 1" 'k_relax\(|k_relax_wl\(|k_relax_wlp\(|k_compact' && bash scripts/ab_counters.sh $O/C4_push C4 "--csr-variant 2" 'k_push|k_pred_pass|k_fold|k_compact'
