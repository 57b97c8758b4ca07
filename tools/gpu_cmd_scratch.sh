mkdir -p gpurun_out
for v in gpu:hostfunc gpu:event gpu:spin host:x gpu:event; do
  p=${v%%:*}; c=${v##*:}
  RHP_REACTOR_COMPLETE=$c RHP_REACTOR_PARSER=$p RHP_REACTOR_STATS=1 timeout -k 10 120 ./libreactorng_amd/bin/burst_test 64 64 9 > gpurun_out/burst_${p}_$c.txt 2>&1 || { cat gpurun_out/burst_${p}_$c.txt | tail; exit 1; }
  echo "== $p $c"; grep -E "req/s" gpurun_out/burst_${p}_$c.txt | tail -9 | awk '{print $0}' | tr '\n' ' '; echo; grep -E "round" gpurun_out/burst_${p}_$c.txt | tail -3
done
