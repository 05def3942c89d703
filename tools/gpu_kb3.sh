set -o pipefail
cd $GRAFT_REPO_ROOT/tools/kbench/_build
export KB_COEF=1
for S in "2 128 64 64 48 1 1 0 1" "2 48 64 64 128 1 1 0 1" "2 48 128 128 16 1 1 0 1" "2 16 128 128 48 1 1 0 1" "2 256 64 64 128 1 1 0 1"; do
  for op in fwd dgrad wgrad; do timeout -k 5 60 ./kbench $op $S 50; done
done
