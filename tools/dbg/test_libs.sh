# GPU box: the GPU tests selected by $K against each library in $LIBS (RQSID_LIB), one pytest per library
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-testlibs}; mkdir -p $O
for lib in $LIBS; do
  n=$(basename $lib .so)
  RQSID_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 300 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread ${K:+-k "$K"} > $O/$n.log 2>&1
  echo "== $n rc=$?"; tail -3 $O/$n.log
done
