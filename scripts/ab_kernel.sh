# A/B of the fused MNIST step kernels on one box: the bare engine loop for each
# variant tree (ab_old = round 1, ab_B / ab_C = bisect variants) and the current tree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
for i in 1 2 3; do
  for d in ab_old; do
    [ -d $d ] || continue
    (cd $d && cp ../scripts/engine_only.py . && timeout -k 10 120 python engine_only.py 2>/dev/null | sed "s/^/$d /") || exit 1
  done
  timeout -k 10 120 python scripts/engine_only.py 2>/dev/null | sed 's/^/new /' || exit 1
done
