#!/bin/bash
# The whole -m gpu suite on the in-tree build, then tools/job_abn.sh ROUNDS LIB...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/abn
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/abn/pytest.log 2>&1 || { tail -40 gpurun_out/abn/pytest.log; exit 1; }
tail -1 gpurun_out/abn/pytest.log
bash tools/job_abn.sh "$@"
