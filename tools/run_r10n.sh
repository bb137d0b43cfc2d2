set -o pipefail
# Full GPU suite with per-test durations, smoke(), and the N = 1 line, on the
# current tree.
O=gpurun_out/r10n
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider --durations=40 > $O/gpu_suite.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench1.json 2> $O/bench1.err
