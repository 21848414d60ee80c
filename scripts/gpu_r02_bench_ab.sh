# r02: headline bench A/B, current library vs scripts/_debug/libcheb_planes.so
set -o pipefail
O=gpurun_out/t12
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_basis_layout.py tests/test_gpu_fused_adam.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && echo PYTEST_OK &&
for i in 1 2 3; do
timeout -k 10 180 python bench.py --steps 2000 --warmup 100 --no-cpu-baseline > $O/bench_new_$i.json 2> $O/bench_new_$i.err &&
CG_LIB_PATH=scripts/_debug/libcheb_planes.so timeout -k 10 180 python bench.py --steps 2000 --warmup 100 --no-cpu-baseline > $O/bench_prev_$i.json 2> $O/bench_prev_$i.err || exit 1
done && echo BENCH_OK
