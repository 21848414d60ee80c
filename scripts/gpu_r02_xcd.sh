# r02: streaming steps with the sample-per-XCD mapping for any N (config R's
# batch of 100): full GPU suite, config R/C2 new vs previous release build
set -o pipefail
O=gpurun_out/t3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 300 python scripts/bench_configs.py R C2 > $O/configs_new.jsonl 2> $O/configs_new.err &&
CG_LIB_PATH=scripts/_debug/libcheb_prev.so timeout -k 10 300 python scripts/bench_configs.py R C2 > $O/configs_prev.jsonl 2> $O/configs_prev.err && echo CONFIGS_OK
