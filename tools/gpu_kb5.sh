# kbench: finalised BN coefficients (KB_COEF=1) vs consumer-side evaluation from the
# statistics, on the op shapes that carry most of the step
set -o pipefail
cd $GRAFT_REPO_ROOT/tools/kbench/_build
for S in "dgrad 2 128 64 64 48 1 1 0 1" "dgrad 2 48 64 64 128 1 1 0 1" "fwd 2 128 64 64 48 1 1 0 1" \
         "fwd 2 48 64 64 128 1 1 0 1" "fwd 2 4 256 256 16 1 1 0 1" "fwd 2 16 256 256 4 1 1 0 1" \
         "wgrad 2 48 64 64 128 1 1 0 1" "wgrad 2 128 64 64 48 1 1 0 1" "dgrad 2 16 128 128 48 1 1 0 1"; do
  a=$(KB_COEF=1 timeout -k 5 60 ./kbench $S 100 | head -1); b=$(timeout -k 5 60 ./kbench $S 100 | head -1)
  echo "$S | coef: $a | stats: $b"
done
