set -o pipefail
mkdir -p gpurun_out/smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke/smoke.log 2>&1 || { tail -20 gpurun_out/smoke/smoke.log; exit 1; }
tail -1 gpurun_out/smoke/smoke.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu-baseline --no-cer > gpurun_out/smoke/torchrun.log 2>&1 || { tail -20 gpurun_out/smoke/torchrun.log; exit 1; }
grep -o '"n_gpus": [0-9]*\|"ms_per_step": [0-9.]*\|"traffic": [0-9a-z]*' gpurun_out/smoke/torchrun.log
