source gpu_step.sh
# what the driver runs at round end, on the final tree
run tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench 300 python -u bench.py
echo done
