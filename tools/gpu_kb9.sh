set -o pipefail
cd $GRAFT_REPO_ROOT/tools/kbench/_build || exit 1
for S in "wgrad 2 48 64 64 128 1 1 0 1" "wgrad 2 128 64 64 48 1 1 0 1" "wgrad 2 16 128 128 48 1 1 0 1" "wgrad 2 256 64 64 128 1 1 0 1"; do
  echo "== $S"; timeout -k 5 60 ./kbench $S 100
done
