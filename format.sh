#!/bin/bash
# Lint (flake8) the Python sources; `--check` exits non-zero on findings.
# C++/HIP sources follow .clang-format (clang-format -i when available).
set -e
cd "$(dirname "$0")"
PY_DIRS="ray_lightning_accelerators_amd ray_lightning tests examples scripts bench.py __graft_entry__.py"
flake8 --config setup.cfg $PY_DIRS
if [ "$1" != "--check" ] && command -v clang-format >/dev/null 2>&1; then
  find ray_lightning_accelerators_amd/csrc \( -name "*.hip" -o -name "*.cpp" -o -name "*.h" \) -print0 | xargs -0 clang-format -i
fi
echo "lint ok"
