"""Backward-weight GEMMs (gemm_tn / conv_wgrad) of a few split plans, results saved to
argv[1]. Run once with MPIT_TN_FUSED=1 (in-kernel split reduction) and once without
(split_reduce launches): tests/test_gemm.py compares the two bit for bit."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from mpit_amd._ext import native
from mpit_amd.ops import conv as C

out = {}
torch.manual_seed(5)
for (M, N, K) in [(802816, 64, 64), (200704, 128, 128), (12544, 512, 2048), (5000, 192, 320)]:
    for dt in (torch.bfloat16, torch.float32):
        y = torch.randn(M, N, device="cuda").to(dt)
        x = torch.randn(M, K, device="cuda").to(dt)
        out[f"tn{M}x{N}x{K}{dt}"] = C.gemm_tn(y, x).cpu()
        base = torch.randn(N, K, device="cuda")
        out[f"tnb{M}x{N}x{K}{dt}"] = C.gemm_tn(y, x, out=base.clone(), beta=1.0).cpu()
m = native()
st = torch.cuda.current_stream().cuda_stream
for (nb, h, c, co) in [(256, 56, 64, 64), (64, 14, 256, 256)]:
    for dt, f32 in ((torch.bfloat16, False), (torch.float32, True)):
        x = torch.randn(nb, h, h, c, device="cuda").to(dt)
        dy = torch.randn(nb, h, h, co, device="cuda").to(dt)
        dw = torch.empty(co, 3, 3, c, device="cuda")
        nws = m.conv_wgrad_ws_floats(0, nb, h, h, c, co, 3, 3, 1, 1)
        ws = torch.empty(max(1, nws), device="cuda")
        m.conv_wgrad(0, st, nb, h, h, c, co, 3, 3, 1, 1, dy.data_ptr(), x.data_ptr(), dw.data_ptr(), ws.data_ptr(),
                     0.0, f32=f32)
        out[f"wg{nb}x{h}x{c}x{co}{f32}"] = dw.cpu()
torch.cuda.synchronize()
torch.save(out, sys.argv[1])
print("saved", len(out))
