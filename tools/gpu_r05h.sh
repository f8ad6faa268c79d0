# round 5, session h: counters of the shipped wide-code kernels (tools/pmc_wide.sh)
# and of the first_seen leg (tools/pmc_sq.sh), on the committed tree
set -o pipefail
bash tools/pmc_wide.sh r05w && bash tools/pmc_sq.sh first_seen r05fs
