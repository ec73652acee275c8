set -u
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests -k "add or golden or smoke or bench_two" > gpurun_out/t_peel.log 2>&1; echo "pytest rc=$? $(tail -1 gpurun_out/t_peel.log)"
bash scripts/ab_bench_only.sh nopeel || exit 1
bash scripts/ab_bench_only.sh nopeel || exit 1
