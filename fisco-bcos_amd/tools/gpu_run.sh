# One gpurun call made of named steps, run in order; the first step that fails, times out or crashes ends
# the call (no retries).  Outputs under gpurun_out/.
#   bash fisco-bcos_amd/tools/gpu_run.sh STEP [STEP ...]
# steps:
#   tests[=PYTEST_K]     the -m gpu suite (or the tests PYTEST_K selects, ',' for ' '), one pytest process
#   file=PATH[::K]       the -m gpu tests of one file (optionally -k K)
#   smoke                __graft_entry__.smoke()
#   bench[=ARGS]         bench.py (default arguments = the driver's default run), ARGS with ',' for ' '
#   profile=WL[,WL...]   rocprofv3 kernel trace + PMC passes per workload (tools/gpu_profile_all.sh)
#   legprof[=LEGS]       rocprofv3 trace + PMC passes of the bench's Merkle / hash legs (tools/gpu_profile_legs.sh)
#   sweep[=ARGS]         tools/small_sweep.py (ARGS with ',' for ' ')
#   exe=PATH[,ARGS]      run a built tool from fisco-bcos_amd/lib (ARGS with ',' for ' ')
#   ab=NAME[,ARGS]       bench.py ARGS with lib_ab/NAME/libbcosgpu.so swapped in (tools/build_ab.sh), then restored
#   py=NAME[,ARGS]       run fisco-bcos_amd/tools/NAME.py (ARGS with ',' for ' '), stdout to gpurun_out/NAME_<step>.json
#   abpy=LIB,NAME[,ARGS] the py step with lib_ab/LIB/libbcosgpu.so swapped in, then restored
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  name=${step%%=*}; arg=""; [ "$name" != "$step" ] && arg=${step#*=}
  log=gpurun_out/step${n}_${name}.log
  case $name in
    tests)
      k=(); [ -n "$arg" ] && k=(-k "${arg//,/ }")
      timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" > $log 2>&1 ;;
    file)
      f=${arg%%::*}; k=(); [ "$f" != "$arg" ] && k=(-k "${arg#*::}")
      k=("${k[@]//,/ }")
      timeout -k 10 900 python3 -u -m pytest $f -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" > $log 2>&1 ;;
    smoke)
      timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $log 2>&1 ;;
    bench)
      timeout -k 10 600 python3 -u bench.py ${arg//,/ } > gpurun_out/bench_${n}.json 2> $log ;;
    profile)
      R=${R:-r05} timeout -k 10 1100 bash fisco-bcos_amd/tools/gpu_profile_all.sh ${arg//,/ } > $log 2>&1 ;;
    legprof)
      R=${R:-r05} timeout -k 10 1200 bash fisco-bcos_amd/tools/gpu_profile_legs.sh ${arg//,/ } > $log 2>&1 ;;
    sweep)
      timeout -k 10 900 python3 -u fisco-bcos_amd/tools/small_sweep.py ${arg//,/ } > gpurun_out/sweep_${n}.json 2> $log ;;
    exe)
      a=${arg//,/ }; timeout -k 10 300 fisco-bcos_amd/lib/$a > $log 2>&1 ;;
    ab)
      v=${arg%%,*}; a=""; [ "$v" != "$arg" ] && a=${arg#*,}
      cp fisco-bcos_amd/lib/libbcosgpu.so /tmp/libbcosgpu.main.so && cp fisco-bcos_amd/lib_ab/$v/libbcosgpu.so fisco-bcos_amd/lib/ && \
      timeout -k 10 600 python3 -u bench.py ${a//,/ } > gpurun_out/ab_${v}_${n}.json 2> $log
      rc0=$?; cp /tmp/libbcosgpu.main.so fisco-bcos_amd/lib/libbcosgpu.so; (exit $rc0) ;;
    abpy)
      v=${arg%%,*}; rest=${arg#*,}; a=${rest//,/ }
      cp fisco-bcos_amd/lib/libbcosgpu.so /tmp/libbcosgpu.main.so && cp fisco-bcos_amd/lib_ab/$v/libbcosgpu.so fisco-bcos_amd/lib/ && \
      timeout -k 10 900 python3 -u fisco-bcos_amd/tools/$a > gpurun_out/ab_${v}_${n}.json 2> $log
      rc0=$?; cp /tmp/libbcosgpu.main.so fisco-bcos_amd/lib/libbcosgpu.so; (exit $rc0) ;;
    py)
      a=${arg//,/ }; timeout -k 10 900 python3 -u fisco-bcos_amd/tools/$a > gpurun_out/${arg%%,*}_${n}.json 2> $log ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "step $n $step rc=$rc"
  tail -c 1500 $log
  [ $rc -eq 0 ] || exit $rc
done
exit 0
