cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/tpw
for t in 8 4 2 16 8; do
  NP_ENC_TPW=$t NP_REC_TPW=$t timeout -k 10 120 python bench.py --no-cpu --steps 20 --warmup 3 > gpurun_out/tpw/t$t.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/tpw/t$t.log').read().strip().split('\n')[-1]); print('tpw $t', d['value'], {k:v['ms'] for k,v in d['kernels'].items()})"
done
