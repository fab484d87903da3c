"""Per-layer timing of VGG-16's 3x3 convolutions (batch 64 by default, channels_last):
our implicit-GEMM kernels (forward, stride-1 backward-data, backward-weight) against
MIOpen's (``F.conv2d`` / ``aten.convolution_backward``) on the same tensors.

    python benchmarks/vgg_layers.py [batch] [bf16|fp32]

One JSON line per layer shape (with its multiplicity in the network) and a totals line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from mpit_amd._ext import native
from mpit_amd.ops import conv as MC

# (H = W, Cin, Cout, multiplicity) of VGG-16's 3x3 / pad 1 / stride 1 layers (not the 3-channel stem)
LAYERS = [(224, 64, 64, 1), (112, 64, 128, 1), (112, 128, 128, 1), (56, 128, 256, 1), (56, 256, 256, 2),
          (28, 256, 512, 1), (28, 512, 512, 2), (14, 512, 512, 3)]


def timeit(fn, it=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    dt = torch.float32 if (len(sys.argv) > 2 and sys.argv[2] == "fp32") else torch.bfloat16
    f32 = dt == torch.float32
    nm = native()
    dev = torch.device("cuda")
    tot = {"ours": 0.0, "miopen": 0.0}
    for hw, cin, cout, mult in LAYERS:
        cl = torch.channels_last
        x = torch.randn(batch, cin, hw, hw, device=dev, dtype=dt).contiguous(memory_format=cl)
        wt = (torch.randn(cout, cin, 3, 3, device=dev, dtype=dt) * 0.05).contiguous(memory_format=cl)
        y = F.conv2d(x, wt, padding=1)
        gy = torch.randn_like(y)
        fl = 2.0 * y.numel() * cin * 9
        t_f = timeit(lambda: F.conv2d(x, wt, padding=1))
        t_d = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, [1, 1], [1, 1], [1, 1], False,
                                                                  [0, 0], 1, [True, False, False]))
        t_w = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, [1, 1], [1, 1], [1, 1], False,
                                                                  [0, 0], 1, [False, True, False]))
        wb, wtt = MC.conv_weights(wt.float().contiguous(memory_format=cl), dgrad=True, dtype=dt)
        d, st = x.device.index, torch.cuda.current_stream().cuda_stream
        yk, dxk = torch.empty_like(y), torch.empty_like(x)
        nws = nm.conv_wgrad_ws_floats(d, batch, hw, hw, cin, cout, 3, 3, 1, 1)
        ws = torch.empty(max(nws, 1), device=dev, dtype=torch.float32)
        dwk = torch.empty(cout, 3, 3, cin, device=dev, dtype=torch.float32)
        k_f = timeit(lambda: nm.conv_fwd(d, st, batch, hw, hw, cin, cout, 3, 3, 1, 1, x.data_ptr(), wb.data_ptr(),
                                         yk.data_ptr(), 0, 0, f32=f32))
        k_d = timeit(lambda: nm.conv_fwd(d, st, batch, hw, hw, cout, cin, 3, 3, 1, 1, gy.data_ptr(), wtt.data_ptr(),
                                         dxk.data_ptr(), 0, 0, f32=f32))
        k_w = timeit(lambda: nm.conv_wgrad(d, st, batch, hw, hw, cin, cout, 3, 3, 1, 1, gy.data_ptr(), x.data_ptr(),
                                           dwk.data_ptr(), ws.data_ptr(), 0.0, f32=f32))
        tf = lambda t: round(fl / t / 1e9, 1)
        print(json.dumps({"hw": hw, "cin": cin, "cout": cout, "mult": mult, "dtype": str(dt)[6:],
                          "ours_ms": [round(k_f, 4), round(k_d, 4), round(k_w, 4)],
                          "miopen_ms": [round(t_f, 4), round(t_d, 4), round(t_w, 4)],
                          "ours_tflops": [tf(k_f), tf(k_d), tf(k_w)],
                          "miopen_tflops": [tf(t_f), tf(t_d), tf(t_w)]}), flush=True)
        tot["ours"] += mult * (k_f + k_d + k_w)
        tot["miopen"] += mult * (t_f + t_d + t_w)
    print(json.dumps({"total_ms": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
