cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for lib in librhp.so librhp_noexact.so; do for x in 0 1; do
RHP_LIB=$PWD/libreactorng_amd/$lib RHP_EXPERIMENT=$x timeout -k 10 120 python bench.py --no-cpu --steps 20 --warmup 3 > gpurun_out/exp3.json 2>/dev/null || exit 1
echo "$lib exp=$x $(python -c "import json;d=json.load(open('gpurun_out/exp3.json'));print(d['value'],d['roofline']['kernel_ms'])")"
done; done
