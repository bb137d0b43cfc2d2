set -o pipefail
# Final check of the round: the max-count worker (automatic schedule added),
# then the full GPU suite and smoke() on the final library.
O=${O:-gpurun_out/r12a}
mkdir -p $O
O=$O/maxcount bash tools/run_r11v.sh || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider --durations=12 > $O/gpu_suite.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.txt 2>&1
