import sys, os, ctypes as C, time
sys.path.insert(0,'ray-tracer-from-scratch_amd')
from rtamd import capi, scenes
import torch
lib=capi.load(os.path.abspath(sys.argv[1])); cfgn=sys.argv[2]; memo=int(sys.argv[3])
dev=torch.device('cuda',0); st=torch.cuda.Stream(dev)
cfg=scenes.CONFIGS[cfgn]; prims=scenes.to_prims(cfg.scene()); arr=(capi.rt_prim*len(prims))(*prims)
cam=capi.camera_init(**scenes.camera_args(cfg.width,cfg.height))
out=torch.empty((cam.height,cam.width,3),device=dev)
h=C.c_void_p(); capi.check(lib.rt_ctx_create(0,C.byref(h))); capi.check(lib.rt_set_scene(h,arr,len(prims)))
lib.rt_set_option(h, capi.RT_OPT_BOX_CACHE, memo)
for _ in range(1050):
    lib.rt_render_device(h,C.byref(cam),0,cam.height,cfg.depth,3,0,0,C.c_void_p(out.data_ptr()),None,C.c_void_p(st.cuda_stream))
torch.cuda.synchronize()
print(cfgn, 'memo', memo, flush=True)
lib.rt_ctx_destroy(h)
