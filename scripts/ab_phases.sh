# Phase stamps (32-64 b32) of the round-1 tree vs the current tree on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
(cd ab_old && mkdir -p gpurun_out && timeout -k 10 120 python ../scripts/mlp_phase_probe.py quick 2>/dev/null | sed 's/^/old /') || exit 1
timeout -k 10 120 python scripts/mlp_phase_probe.py quick 2>/dev/null | sed 's/^/new /' || exit 1
