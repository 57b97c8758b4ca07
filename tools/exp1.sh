cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_exp1.log 2>&1 && echo PYTEST_OK \
&& for f in 0 1 2 3; do RHP_DFA_FLAGS=$f timeout -k 10 120 python bench.py --no-cpu --steps 30 --warmup 5 > gpurun_out/exp1_f$f.json 2>/dev/null || exit 1; echo "flags=$f $(python -c "import json;d=json.load(open('gpurun_out/exp1_f$f.json'));print(d['value'],d['roofline']['kernel_ms'])")"; done
