cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK && \
VARIANTS="0 52 49 50 51 53 0 52" bash tools/vsweep.sh s1
