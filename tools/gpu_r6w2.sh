set -u
mkdir -p gpurun_out
: > gpurun_out/r6w2_ab.txt
for r in 1 2 3; do
  for v in ilp noilp; do
    if [ $v = noilp ]; then L="LD_LIBRARY_PATH=probes/noilp"; else L="X=1"; fi
    env $L timeout -k 10 120 tools/dropin_latency 4000 > gpurun_out/r6w2_$v.json 2>&1 || { tail -5 gpurun_out/r6w2_$v.json; exit 1; }
    echo "$r $v $(cat gpurun_out/r6w2_$v.json)" >> gpurun_out/r6w2_ab.txt
  done
done
cat gpurun_out/r6w2_ab.txt
