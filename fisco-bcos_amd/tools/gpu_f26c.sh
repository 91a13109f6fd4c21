# fe26 cooperative kernel: parity variants, then C2 with each field
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ecc.py -m gpu -x -v --timeout 300 --timeout-method thread -k "variants or synthetic or recover" > gpurun_out/pytest_f26c.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|Error" gpurun_out/pytest_f26c.log | tail -14; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_f26c.log; exit $rc; }
for f in 1 0; do
  BCOSGPU_K1_F26=$f timeout -k 10 200 python3 bench.py --steps 1000 --warmup 20 --warm-seconds 1 --legs= --no-cpu-baseline --no-merkle --no-extras > gpurun_out/bench_c2_f26_$f.json 2> gpurun_out/bench_c2_f26_$f.err || { tail -20 gpurun_out/bench_c2_f26_$f.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_c2_f26_$f.json'));print('f26=$f', d['value'], d['roofline']['kernel'], d['roofline']['kernel_ms'])"
done
