set -u; export TMPDIR=/tmp; O=gpurun_out/r1b_s6; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python tools/opt_ab.py --option ROW_ORDER --values 0,1 --configs c1,c2 --precisions path64,f32 && \
timeout -k 10 200 python tools/ab.py --a ray-tracer-from-scratch_amd/lib/librt_amd.so --b ray-tracer-from-scratch_amd/lib/ab/prio1.so --more ray-tracer-from-scratch_amd/lib/ab/prio2.so --configs c2,c3 --precisions path64,f32 && \
timeout -k 10 200 python tools/wave_times.py --lib ray-tracer-from-scratch_amd/lib/ab/wt.so --setups c2:4:path64,c2:4:f32 --save $O/maps.json
