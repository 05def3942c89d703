set -o pipefail
cd $GRAFT_REPO_ROOT/tools/kbench/_build || exit 1
L2="2 16 512 512 16 5 2 2 1"
for d in 0 1 2 4 3 5 6 7; do
  echo "== dbg=$d"; KB_STAMPS_DOWN=1 ISG_S2W_DBG=$d timeout -k 5 60 ./kbench wgrad $L2 50 || exit 1
done
echo "== 1024 WGs"; KB_STAMPS_DOWN=1 ISG_S2W_WGS=1024 timeout -k 5 60 ./kbench wgrad $L2 50 || exit 1
