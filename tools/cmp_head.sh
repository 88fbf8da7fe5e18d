cd $GRAFT_REPO_ROOT
bash tools/exp_one.sh head base head base || exit 1
ARGS="--config 2" TAG=c2_ bash tools/exp_one.sh head base head base || exit 1
ARGS="--n-wanted 512 --k-wanted 256 --erase 200" TAG=nq2_ bash tools/exp_one.sh head base || exit 1
ARGS="--n-wanted 2048 --k-wanted 256 --erase 1000 --batch 512" TAG=nq8_ bash tools/exp_one.sh head base || exit 1
