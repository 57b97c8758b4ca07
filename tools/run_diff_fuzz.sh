#!/bin/bash
# Differential fuzz of the oracle restatement against the compiled reference
# (dev container only: needs oracle/_ref, built from /root/reference).
# usage: tools/run_diff_fuzz.sh <batches-per-process> <requests-per-batch> <processes> > log
set -e
cd "$(dirname "$0")/.."
make -s -C oracle ref
B=${1:-400}; N=${2:-25000}; P=${3:-4}
echo "diff_fuzz: $P processes x $B batches x $N requests (configs 100/101/3/5/2 x max_headers 0/1/2/4/16/32, phr + http)"
pids=()
for s in $(seq 1 "$P"); do
  ( /usr/bin/time -f "seed $((100 + s)): %e s" oracle/_ref/diff_fuzz "$B" "$N" $((100 + s)) ) > /tmp/rhp_df_$s.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=1; done
for s in $(seq 1 "$P"); do cat /tmp/rhp_df_$s.log; done
exit $rc
