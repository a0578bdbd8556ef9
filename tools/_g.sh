set -u; export TMPDIR=/tmp; O=gpurun_out/${S:-x}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${K:+-k "$K"} > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python tools/ab.py --a ray-tracer-from-scratch_amd/lib/ab/prev.so --b ray-tracer-from-scratch_amd/lib/librt_amd.so ${MORE:+--more $MORE} --configs ${CFGS:-c1,c2} --precisions ${PRECS:-path64,f32} || exit 1
if [ -n "${OPT:-}" ]; then timeout -k 10 200 python tools/opt_ab.py $OPT || exit 1; fi
if [ -n "${WT:-}" ]; then timeout -k 10 200 python tools/wave_times.py --lib ray-tracer-from-scratch_amd/lib/ab/wt.so $WT || exit 1; fi
