# r02: the planes-layout GPU tests on the current tree
set -o pipefail
O=gpurun_out/t13
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_basis_layout.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && echo PYTEST_OK
