# Build a timing-probe copy of libxrs.so from the product sources with one
# sed edit applied (probe/ is git-ignored; the product library never holds
# probe code).   bash scripts/build_probe.sh NAME 'SED-EXPRESSION' [FILE]
set -e
NAME=$1; EXPR=$2; FILE=${3:-xrs_rectify.hip}
R=$(cd "$(dirname "$0")/.." && pwd)
D=$R/probe/$NAME; rm -rf $D; mkdir -p $D/pkg/csrc $D/pkg/lib
ln -s $R/include $D/include
cp $R/xcube-resampling_amd/csrc/* $D/pkg/csrc/
sed -i "$EXPR" $D/pkg/csrc/$FILE
if cmp -s $D/pkg/csrc/$FILE $R/xcube-resampling_amd/csrc/$FILE; then echo "probe $NAME: sed changed nothing" >&2; exit 1; fi
make -s -C $D/pkg/csrc -j4 >/dev/null
echo $D/pkg/lib/libxrs.so
