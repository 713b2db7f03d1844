set -u
bash tools/ab_run.sh > gpurun_out/r4f_ab.txt 2>&1; echo AB_EXIT $? >> gpurun_out/r4f_ab.txt
PROBE_CHECK=1 timeout -k 10 300 python tools/probe_ab.py probes/new.so probes/fold.so probes/new.so probes/fold.so > gpurun_out/r4f_fold.txt 2>&1 || exit 1
PROBE_CHECK=1 timeout -k 10 300 python tools/probe_ab.py probes/q0.so@quad probes/q1.so@quad probes/q2.so@quad > gpurun_out/r4f_quad.txt 2>&1 || exit 1
NO_TDB=1 REPS=1000 timeout -k 10 300 python tools/bench_dropin_latency.py > gpurun_out/r4f_dropin.json 2>&1 || exit 1
PASSES="sqA sqB" bash tools/profile.sh r4f_new --blocks 65536 --iters 2 --which encode --lib probes/new.so > /dev/null 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_probe_decoders.py -x -q -p no:cacheprovider --timeout 700 --timeout-method thread > gpurun_out/r4f_probe.txt 2>&1; echo PROBE_EXIT $? >> gpurun_out/r4f_probe.txt
PROBE_CHECK=1 timeout -k 10 300 python tools/probe_ab.py probes/replay.so > gpurun_out/r4f_replay.txt 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && NO_TDB=1 REPS=300 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4f_dropin -o dropin --output-format csv -- python3 tools/bench_dropin_latency.py > gpurun_out/r4f_dropin_rocprof.txt 2>&1
