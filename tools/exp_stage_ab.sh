set -e
mkdir -p gpurun_out/exp1
for v in default nogen notw; do
  if [ $v = default ]; then unset FGP_LIB_PATH; else export FGP_LIB_PATH=$PWD/fastgaussianprocesses_amd/_lib/exp/libfgp_$v.so; fi
  timeout -k 10 200 python -u tools/stage_times.py --tag $v >> gpurun_out/exp1/times.jsonl 2> gpurun_out/exp1/err_$v.log
done
cat gpurun_out/exp1/times.jsonl
