for i in 1 2; do for v in 0 1; do for ops in 1 2 3; do
  echo "v=$v ops=$ops $(timeout -k 10 60 fisco-bcos_amd/lib_ab/triobench_$v 250 32 $ops | tail -1)" || exit 1
done; done; done
