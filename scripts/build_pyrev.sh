# An A/B arm of the whole package from a git revision — host code (Python)
# and its library, built from that revision's sources (build_rev.sh):
# probe/NAME/root/xcube_resampling_amd (gpu_rect_ab4.sh puts it first on the path).
#   bash scripts/build_pyrev.sh NAME REV
set -e
NAME=$1; REV=$2
R=$(cd "$(dirname "$0")/.." && pwd)
bash $R/scripts/build_rev.sh $NAME $REV > /dev/null
D=$R/probe/$NAME/root; mkdir -p $D
git -C $R archive $REV xcube-resampling_amd | tar -x -C $D --exclude='*/csrc/*'
mkdir -p $D/xcube-resampling_amd/lib
cp $R/probe/$NAME/pkg/lib/libxrs.so $D/xcube-resampling_amd/lib/
ln -s xcube-resampling_amd $D/xcube_resampling_amd
echo $D
