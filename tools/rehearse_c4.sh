#!/bin/bash
# bench.py's N > 1 flow at the full C4 size with 2 ranks sharing the box's GPU
# over gloo (a flow / time / memory check of the partition code at the scale
# the driver's multi-GPU run uses; times are not a measurement).
# Usage: tools/rehearse_c4.sh <strategy> [world] [extra bench.py args]
S=${1:?strategy}; W=${2:-2}; shift; shift; EXTRA="$*"
mkdir -p gpurun_out
LOG=gpurun_out/rehearse_c4_$S
rm -rf $LOG; mkdir -p $LOG
PORT=$((20000 + RANDOM % 20000))
START=$(date +%s)
# heartbeat: the ranks print nothing until their line
( while true; do sleep 45; echo "  ... $(( $(date +%s) - START )) s";
  tail -3 $LOG/*/*/0/stderr.log 2>/dev/null | grep -E "bench|dist"; done ) &
HB=$!
SLDM_DIST_TRACE=${TRACE:-0} timeout -k 10 900 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node=$W --master-addr=127.0.0.1 --master-port=$PORT --log-dir=$LOG --redirects=3 \
  bench.py --gpus $W --config c4 --steps 2 --warmup 1 --dist-backend gloo --strategy $S $EXTRA \
  > $LOG/launcher.log 2>&1
rc=$?
kill $HB 2>/dev/null
echo "strategy $S rc=$rc wall=$(( $(date +%s) - START )) s"
grep -h '^{' $LOG/*/*/0/stdout.log 2>/dev/null | head -1 | cut -c1-600
[ $rc -ne 0 ] && tail -20 $LOG/launcher.log && find $LOG -name "*.log" -path "*/0/*" -exec tail -20 {} \;
exit $rc
