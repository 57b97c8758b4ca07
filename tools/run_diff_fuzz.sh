#!/bin/bash
# Differential fuzz of the oracle restatement against the compiled reference
# (dev container only: needs oracle/_ref, built from /root/reference).
# usage: tools/run_diff_fuzz.sh <batches-per-process> <requests-per-batch> <processes> > log
# Every process prints its own "diff_fuzz OK: ..." line (or the first mismatch);
# the script fails if any process fails.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
make -s -C oracle ref || exit 1
B=${1:-400}; N=${2:-25000}; P=${3:-4}
echo "diff_fuzz: $P processes x $B batches x $N requests (configs 100/101/3/5/2 x max_headers 0/1/2/4/16/32, phr + http)"
echo "host: $(uname -m), $(nproc) CPUs; started $(date -u +%Y-%m-%dT%H:%M:%SZ)"
pids=()
for s in $(seq 1 "$P"); do
  (
    t0=$(date +%s.%N)
    oracle/_ref/diff_fuzz "$B" "$N" $((100 + s))
    rc=$?
    t1=$(date +%s.%N)
    echo "seed $((100 + s)): exit $rc, $(awk -v a="$t0" -v b="$t1" 'BEGIN{printf "%.1f", b-a}') s"
    exit $rc
  ) > /tmp/rhp_df_$s.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=1; done
for s in $(seq 1 "$P"); do cat /tmp/rhp_df_$s.log; done
total=$(awk '/diff_fuzz OK:/{n += $3} END{print n + 0}' /tmp/rhp_df_*.log)
echo "total requests compared: ${total:-0}; exit $rc; finished $(date -u +%Y-%m-%dT%H:%M:%SZ)"
rm -f /tmp/rhp_df_*.log
exit $rc
