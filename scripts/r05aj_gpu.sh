#!/bin/bash
# Round 5, session aj: rehearsal of the N > 1 bench flow on one GPU (all
# ranks on GPU 0: copy exchange instead of RCCL) -- the child process, the
# host-direct headline loop, the gather leg, the checks -- at N = 2 and 8,
# under the launcher and under torchrun.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05aj
mkdir -p $OUT
for n in 2 8; do
  timeout -k 10 400 python bench.py --gpus $n --same-device > $OUT/bench_n$n.log 2>&1 || { echo "n=$n failed"; tail -20 $OUT/bench_n$n.log; exit 1; }
  python3 -c "
import json
t=open('$OUT/bench_n$n.log').read(); d=json.loads(t[t.index('{\"metric'):].split('\n')[0])
print('n=$n', d['value'], d['ms_per_step'], 'dev', d['device_resident_mrays_s'], 'ok', d['last_frame_equals_one_context'], 'other', json.dumps(d.get('other_delivery')))"
done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --same-device > $OUT/torchrun_n2.log 2>&1 || { echo "torchrun failed"; tail -20 $OUT/torchrun_n2.log; exit 1; }
grep -c '"metric"' $OUT/torchrun_n2.log
