# Build an A/B arm of libxrs.so from the product sources of a git revision
# (probe/ is git-ignored; the product library never holds probe code).
#   bash scripts/build_rev.sh NAME REV      -> probe/NAME/pkg/lib/libxrs.so
set -e
NAME=$1; REV=$2
R=$(cd "$(dirname "$0")/.." && pwd)
D=$R/probe/$NAME; rm -rf $D; mkdir -p $D/pkg/csrc $D/pkg/lib $D/include
for f in $(git -C $R ls-tree --name-only $REV xcube-resampling_amd/csrc/); do
  git -C $R show $REV:$f > $D/pkg/csrc/$(basename $f)
done
git -C $R show $REV:include/xrs.h > $D/include/xrs.h
make -s -C $D/pkg/csrc -j4 >/dev/null
echo $D/pkg/lib/libxrs.so
