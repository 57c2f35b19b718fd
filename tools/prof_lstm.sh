cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/bench_lstm.py > gpurun_out/lstm_micro.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lstm -o kt --output-format csv -- python tools/bench_lstm.py > /dev/null 2>&1 || exit 2
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum -d gpurun_out/prof_lstm -o pmc1 --output-format csv -- python tools/bench_lstm.py > /dev/null 2>&1 || exit 3
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES -d gpurun_out/prof_lstm -o pmc2 --output-format csv -- python tools/bench_lstm.py > /dev/null 2>&1 || exit 4
echo done
