set -u; export TMPDIR=/tmp; O=gpurun_out/r1b_s7; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python tools/opt_ab.py --option MIRROR_BINS --values 0,1 --configs c1,c2 --precisions path64,f32,f64
