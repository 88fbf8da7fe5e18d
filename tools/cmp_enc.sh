cd $GRAFT_REPO_ROOT
bash tools/gpu_check_quick.sh || exit 1
ARGS="--n-wanted 1200 --erase 400" TAG=v1200_ bash tools/exp_one.sh head base || exit 1
