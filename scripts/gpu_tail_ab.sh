# r02 A/B on one box: the backward's tail slab reduction (config B bench) and
# the streaming last step with the fused contraction (configs C2, R), new
# library vs the previous release build (scripts/_debug/libcheb_prev.so)
set -o pipefail
O=gpurun_out/t2
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_tail_reduce.py tests/test_gpu_fused_adam.py tests/test_gpu_large.py tests/test_gpu_model.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && echo PYTEST_OK &&
for i in 1 2; do
timeout -k 10 180 python bench.py --steps 2000 --warmup 100 --no-cpu-baseline > $O/bench_new_$i.json 2> $O/bench_new_$i.err &&
CG_LIB_PATH=scripts/_debug/libcheb_prev.so timeout -k 10 180 python bench.py --steps 2000 --warmup 100 --no-cpu-baseline > $O/bench_prev_$i.json 2> $O/bench_prev_$i.err || exit 1
done && echo BENCH_OK &&
timeout -k 10 300 python scripts/bench_configs.py C2 R > $O/configs_new.jsonl 2> $O/configs_new.err &&
CG_LIB_PATH=scripts/_debug/libcheb_prev.so timeout -k 10 300 python scripts/bench_configs.py C2 R > $O/configs_prev.jsonl 2> $O/configs_prev.err && echo CONFIGS_OK
