cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for x in 0 1 3 2; do for w in 16 4; do
RHP_EXPERIMENT=$x RHP_WAVES=$w timeout -k 10 120 python bench.py --no-cpu --steps 20 --warmup 3 > gpurun_out/exp2_x${x}_w$w.json 2>/dev/null || exit 1
echo "exp=$x waves=$w $(python -c "import json;d=json.load(open('gpurun_out/exp2_x${x}_w$w.json'));print(d['value'],d['roofline']['kernel_ms'])")"
done; done
