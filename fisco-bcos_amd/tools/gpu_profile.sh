# Runs the GPU test suite and the rocprofv3 passes (kernel trace + separate PMC passes) on the MI355X box.
set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_all.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_all.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o r01 -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch -o r01 -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write -o r01 -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_write.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/prof/sq -o r01 -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_sq.log 2>&1
echo "prof rc=$?"
tail -3 gpurun_out/pytest_all.log
find gpurun_out/prof -name "*.csv" | head -20
