# Windowed kernel profile of the burst-sized prefill (5 sequences, 380 rows) on the final tree.
set -o pipefail
TAG=r4burst STAGES=profpf TOKENS=380 SEQS=5 REPS=5 bash scripts/gpu/stages.sh
