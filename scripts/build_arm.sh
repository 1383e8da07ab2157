# Build an A/B arm of libxrs.so: the working tree's sources with one file
# replaced (probe/ is git-ignored; the product library never holds probe code).
#   bash scripts/build_arm.sh NAME CSRC_FILE REPLACEMENT   -> probe/NAME/pkg/lib/libxrs.so
set -e
NAME=$1; FILE=$2; REPL=$3
R=$(cd "$(dirname "$0")/.." && pwd)
D=$R/probe/$NAME; rm -rf $D; mkdir -p $D/pkg/csrc $D/pkg/lib
ln -s $R/include $D/include
cp $R/xcube-resampling_amd/csrc/* $D/pkg/csrc/
cp $REPL $D/pkg/csrc/$FILE
make -s -C $D/pkg/csrc -j4 >/dev/null
echo $D/pkg/lib/libxrs.so
