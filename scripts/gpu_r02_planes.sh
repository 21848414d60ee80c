# r02: planes basis layout for the ResGNN hidden layers (streaming path):
# full GPU suite, config R/C2, headline bench
set -o pipefail
O=gpurun_out/t5
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 300 python scripts/bench_configs.py R C2 > $O/configs_new.jsonl 2> $O/configs_new.err && echo CONFIGS_OK &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && echo BENCH_OK
