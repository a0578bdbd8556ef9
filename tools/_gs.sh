set -u
export TMPDIR=/tmp
O=gpurun_out/${S:-x}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${K:+-k "$K"} > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/opt_ab.py ${AB:---option TILE_BINS --values 0,1 --configs c1,c2 --precisions path64,f64,mixed} > $O/ab.jsonl 2>$O/ab.err; rc=$?
cat $O/ab.jsonl; tail -3 $O/ab.err; exit $rc
