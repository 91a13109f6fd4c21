# fe26 throughput kernel: occupancy 1 vs 2, and PMC (instructions, scratch traffic) for each field
mkdir -p gpurun_out/f26
export TMPDIR=/tmp
B="python3 bench.py --workload c4 --steps 10 --warmup 2 --warm-seconds 0 --legs= --no-cpu-baseline --no-merkle --no-extras"
for cfg in "1 1" "1 2" "0 2"; do
  set -- $cfg
  BCOSGPU_K1_F26=$1 BCOSGPU_TXV_OCC=$2 timeout -k 10 200 python3 bench.py --workload c4 --steps 30 --warmup 3 --warm-seconds 1 --legs= --no-cpu-baseline --no-merkle --no-extras > gpurun_out/f26/b_$1_$2.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/f26/b_$1_$2.json'));print('f26=$1 occ=$2', round(d['value']/1e6,2), d['roofline']['kernel'], round(d['roofline']['kernel_ms'],3))"
done
for f in 1 0; do
  BCOSGPU_K1_F26=$f timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/f26/sq$f -o run -- $B > gpurun_out/f26/sq$f.log 2>&1 || exit 1
  BCOSGPU_K1_F26=$f timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/f26/fe$f -o run -- $B > gpurun_out/f26/fe$f.log 2>&1 || exit 1
  BCOSGPU_K1_F26=$f timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/f26/wr$f -o run -- $B > gpurun_out/f26/wr$f.log 2>&1 || exit 1
done
echo ok
