# Build a timing-probe copy of libxrs.so from the product sources with a
# Python string replacement applied (multi-line edits sed cannot express;
# probe/ is git-ignored).   bash scripts/build_probe_py.sh NAME FILE OLD NEW
set -e
NAME=$1; FILE=$2; OLD=$3; NEW=$4
R=$(cd "$(dirname "$0")/.." && pwd)
D=$R/probe/$NAME; rm -rf $D; mkdir -p $D/pkg/csrc $D/pkg/lib
ln -s $R/include $D/include
cp $R/xcube-resampling_amd/csrc/* $D/pkg/csrc/
python3 - "$D/pkg/csrc/$FILE" "$OLD" "$NEW" <<'PY'
import sys
p, old, new = sys.argv[1], sys.argv[2].encode().decode("unicode_escape"), sys.argv[3].encode().decode("unicode_escape")
s = open(p).read()
if old not in s:
    sys.exit("probe: OLD text not found")
open(p, "w").write(s.replace(old, new))
PY
make -s -C $D/pkg/csrc -j4 >/dev/null
echo $D/pkg/lib/libxrs.so
