import sys, time, ctypes as C
sys.path.insert(0, '.')
import numpy as np
import cudavolumerenderer_amd as cvr
lib = cvr.load()
lib.cvr_debug_counters.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
s = cvr.Scene.synthetic('manix', 0, (64, 58, 64))
for W, it, grid in [(32, 1, 1), (64, 1, 1), (64, 2, 0), (128, 4, 0)]:
    ctx = cvr.Context(0, 'regenerationSK')
    ctx.set_option(cvr.OPT_SCHEDULER, 2)
    ctx.set_option(cvr.OPT_GRID, grid)
    ctx.set_medium(s.medium)
    iv, r2v = cvr.default_camera(W, W)
    ctx.set_camera(iv, r2v, (W, W))
    ctx.init(); ctx.set_resolution(W, W); ctx.set_iterations(it)
    ctx.clear_output(); t = time.time(); ctx.launch_render(); st = ctx.stats()
    out = (C.c_uint64 * 16)(); lib.cvr_debug_counters(ctx._h, out)
    print(W, it, grid, 'ms', round((time.time() - t) * 1e3, 1), 'paths', st.paths, 'steps', st.steps, 'esc', st.escaped, 'dbg', list(out)[:4], flush=True)
