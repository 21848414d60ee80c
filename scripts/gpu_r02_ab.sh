# r02: streaming SpMM rows: next batch of col/val issued behind the gathers (row_spmm), A/B vs
# the library before it (scripts/_debug/libcheb_planes.so) on configs R, C2, D
set -o pipefail
O=gpurun_out/t10
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_basis_layout.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && echo PYTEST_OK &&
for i in 1 2; do
timeout -k 10 300 python scripts/bench_configs.py R C2 D > $O/new_$i.jsonl 2> $O/new_$i.err &&
CG_LIB_PATH=scripts/_debug/libcheb_planes.so timeout -k 10 300 python scripts/bench_configs.py R C2 D > $O/prev_$i.jsonl 2> $O/prev_$i.err || exit 1
done && echo AB_OK
