# round 5 final tree, part 2: per-leg kernel traces and PMC traffic of every
# BASELINE workload (tools/profile_r02.sh), then the issue-side counters
# (tools/pmc_sq.sh) of the same workloads and the first_seen leg
set -o pipefail
P=${TAG:-r05p}
bash tools/profile_r02.sh $P cfg2 cfg3 cfg4 cfg5 || { echo profile-failed; exit 1; }
for w in cfg2 cfg3 cfg4 cfg5 first_seen; do
  bash tools/pmc_sq.sh $w ${P}sq || { echo pmc-$w-failed; exit 1; }
done
echo final2-done
