#!/bin/bash
# End-of-session GPU run: parity tests, smoke, headline bench, kernel-trace summaries,
# band-KKT PMC passes, headline PMC traffic passes.  Each GPU step has its own time
# limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/gpu_check.sh || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
bash scripts/gpu_bandpmc.sh || exit $?
bash scripts/gpu_profile.sh || exit $?
