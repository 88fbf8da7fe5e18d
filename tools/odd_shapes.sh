#!/bin/bash
# Payload sizes whose chunk counts make shard rows 2- or 4-byte aligned (DESIGN
# §6): the config-3 shape with 1,000,000- and 1,000,001-byte payloads, the
# reference bench's 2,000 validators x 10 MB, 100 validators with 1,000,003.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/odd
run() { tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 2 "$@" > gpurun_out/odd/$tag.log 2>&1 || { tail -5 gpurun_out/odd/$tag.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/odd/$tag.log').read().strip().split('\n')[-1])
c=d['config']; print('$tag', 'n', c['n'], 'k', c['k'], 'GiB/s', d['value'], {k:(v['ms'], v['frac']) for k,v in d['kernels'].items()}, 'ok', d['roundtrip_ok'])"
}
run c3_1000000 --payload 1000000 &&
run c3_1000001 --payload 1000001 &&
run vc2000_10MB --n-wanted 2000 --batch 100 --payload 10000000 --erase 667 &&
run vc100_1000003 --n-wanted 100 --batch 1024 --payload 1000003 --erase 34
