# round 5, session c: issue-side counters (VALU, LDS, SALU, branch) of the
# first_seen leg (matapply_bsr<10,lds> and the compiled k20_r20 kernel)
set -o pipefail
bash tools/pmc_sq.sh first_seen r05c
