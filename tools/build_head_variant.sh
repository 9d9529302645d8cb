# Builds the library of a git revision (default HEAD) as variant <tag> (A/B baseline)
# usage: bash tools/build_head_variant.sh <tag> [rev]
set -e
TAG=${1:-prev}; REV=${2:-HEAD}
R=$(cd "$(dirname "$0")/.." && pwd)
rm -rf /tmp/mr_wt && git -C "$R" worktree add -f /tmp/mr_wt "$REV" > /dev/null 2>&1
(cd /tmp/mr_wt && python -m marshrutka_amd.build --variant "$TAG" > /dev/null 2>&1)
mkdir -p "$R/marshrutka_amd/lib/variants/$TAG"
cp /tmp/mr_wt/marshrutka_amd/lib/variants/$TAG/libmarshrutka_pf.so "$R/marshrutka_amd/lib/variants/$TAG/"
git -C "$R" worktree remove --force /tmp/mr_wt
echo "variant $TAG = $REV"
