set -o pipefail
cd $GRAFT_REPO_ROOT/tools/kbench/_build || exit 1
L2="2 16 512 512 16 5 2 2 1"
for F in "" "ISG_TWA_FORCE=1"; do
 for d in 0 1 2 4 8 5; do
  echo "== wgrad L2 $F dbg=$d"; env $F ISG_TW_DBG=$d timeout -k 5 60 ./kbench wgrad $L2 50 || exit 1
 done
done
echo "== fwd L2"; timeout -k 5 60 ./kbench fwd $L2 50 || exit 1
echo "== fwd L2 s2k5"; ISG_S2K5=1 timeout -k 5 60 ./kbench fwd $L2 50 || exit 1
echo "== dgrad L2"; timeout -k 5 60 ./kbench dgrad $L2 50 || exit 1
for S in "2 48 64 64 128 1 1 0 1" "2 128 64 64 48 1 1 0 1" "2 256 64 64 128 1 1 0 1" "2 16 128 128 48 1 1 0 1"; do
  echo "== wgrad $S"; timeout -k 5 60 ./kbench wgrad $S 100 || exit 1
done
