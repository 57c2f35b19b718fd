#!/bin/bash
# Kernel-time stats and HBM traffic of the bench step, for profiles/.
# Run on the GPU box from the repo root:  bash tools/profile_round.sh r1
# Three separate rocprofv3 runs: --kernel-trace --stats, then one --pmc pass
# per TCC counter (FETCH_SIZE, WRITE_SIZE); every GPU step has its own limit.
set -o pipefail
tag=${1:?tag}
out=gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
cmd=(python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-cer)
pmc=(python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-cer)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- "${cmd[@]}" \
    > "$out/trace.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$out/fetch" -o run --output-format csv -- "${pmc[@]}" \
    > "$out/fetch.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$out/write" -o run --output-format csv -- "${pmc[@]}" \
    > "$out/write.log" 2>&1 || exit $?
python3 tools/pmc_traffic.py --fetch "$out/fetch" --write "$out/write" --match "conv3x3_direct_kernel<[0-9]+, [0-9]+, [0-9]+, false|gemm_nt_kernel<([0-9]+, ){5}2, [48](, (false|true))*>|conv3x3_fwd_rows_kernel|conv3x3_fwd_rows_co_kernel|conv12_fwd_rows_kernel" \
    --desc "conv1-conv8 forward launches (conv12_fwd_rows_kernel conv1 -> conv2, conv3x3_fwd_rows_co_kernel conv3-conv5, gemm_nt_kernel<..., A_IM2COL, NW> conv6-conv8)" \
    --command "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE -- ${pmc[*]}" --out "$out/pmc_conv.json" || exit $?
find "$out/trace" -name "*kernel_stats.csv" -exec cp {} "$out/kernel_stats.csv" \;
python3 tools/conv_table.py --trace "$out/trace" --fetch "$out/fetch" --write "$out/write" --out "$out/conv_layers.md" || exit $?
python3 tools/kernel_table.py --trace "$out/trace" --fetch "$out/fetch" --write "$out/write" --steps 7 --pmc-steps 2 \
    --out "$out/kernel_table.md" || exit $?
grep '^{' "$out/trace.log" | tail -1 > "$out/bench_under_trace.json"
true
