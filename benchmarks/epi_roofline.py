"""Roofline of the backward-data NT GEMMs with the BN-reduction epilogue (EPI_BNRED, the
``epi=2`` calls of profiles/gemm_calls_*), standalone, against copy kernels moving the same
read / write mix — and the same call with the layer's weight-gradient GEMM (gemm_tn)
running concurrently on a second stream, as it does inside the training step.

Per shape and dtype (fp32 = fp16x3 split GEMMs, bf16):
  plain       C = A.B^T                                   bytes A + B + C
  bnred       + dz = C*mask, (sum dz, sum dz (x - mean))  + x + mask bits
  bnred_cin   + C += Cin*cmask (the parked residual grad) + Cin + cmask bits
  copy_2r1w   torch.add(x, cin, out=c) over M*N           the achievable 2-read/1-write rate
  side        bnred_cin on stream 1 || gemm_tn (the layer's wgrad) on stream 2: wall time of
              both, and each alone

    python benchmarks/epi_roofline.py [fp32|bf16 ...]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

SHAPES = [(802816, 256, 64), (802816, 64, 256), (802816, 256, 128), (200704, 512, 128), (200704, 128, 512),
          (50176, 1024, 256), (50176, 256, 1024)]


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
    return s.elapsed_time(e) / it * 1e3  # us


def main():
    from mpit_amd._ext import native
    from mpit_amd.ops import conv as C

    m = native()
    dev = torch.device("cuda")
    s0 = torch.cuda.current_stream()
    s1 = torch.cuda.Stream()
    dts = [a for a in sys.argv[1:] if a in ("fp32", "bf16")] or ["fp32", "bf16"]
    for dn in dts:
        dt = torch.float32 if dn == "fp32" else torch.bfloat16
        f32 = dt == torch.float32
        es = 4 if f32 else 2
        for M, N, K in SHAPES:
            torch.manual_seed(0)
            a = torch.randn(M, K, device=dev).to(dt)
            b = (torch.randn(N, K, device=dev) * 0.05).to(dt)
            c = torch.empty(M, N, device=dev, dtype=dt)
            x = torch.randn(M, N, device=dev).to(dt)
            cin = torch.randn(M, N, device=dev).to(dt)
            mask = torch.randint(0, 256, (M * N // 8,), dtype=torch.uint8, device=dev)
            cmask = torch.randint(0, 256, (M * N // 8,), dtype=torch.uint8, device=dev)
            mean = torch.randn(N, device=dev)
            nt = m.gemm_nt_tiles(M)
            part = torch.empty(nt * 2 * N, dtype=torch.float32, device=dev)
            keep = []
            if f32:
                bp = C.f16_planes(b.contiguous(), C.bound_of_value(torch.linalg.vector_norm(b, float("inf"))))
                C.set_amax(a, C.bound_of_value(torch.linalg.vector_norm(a, float("inf"))))
                kw = C._split_kw(a, bp, True, keep)
                bb = bp
            else:
                kw, bb = {}, b
            st = s0.cuda_stream
            red = dict(red_part=part.data_ptr(), red_x=x.data_ptr(), red_mask=mask.data_ptr(), red_mean=mean.data_ptr())

            def nt_call(stream=st, **extra):
                m.gemm_nt(0, stream, M, N, K, a.data_ptr(), K, bb.data_ptr(), K, c.data_ptr(), N, 0, f32=f32,
                          **kw, **extra)

            base = (M * K + N * K + M * N) * es
            xb, mb = M * N * es, M * N // 8
            row = {"dtype": dn, "M": M, "N": N, "K": K}
            for name, extra, by in (("plain", {}, base), ("bnred", red, base + xb + mb),
                                    ("bnred_cin", dict(red, cin=cin.data_ptr(), cmask=cmask.data_ptr()),
                                     base + 2 * xb + 2 * mb)):
                t = timeit(lambda: nt_call(**extra))
                row[name + "_us"] = round(t, 1)
                row[name + "_TBs"] = round(by / t / 1e6, 2)
            t = timeit(lambda: torch.add(x, cin, out=c))
            row["copy_2r1w_TBs"] = round(3 * xb / t / 1e6, 2)
            t = timeit(lambda: c.copy_(x))
            row["copy_1r1w_TBs"] = round(2 * xb / t / 1e6, 2)
            # the layer's weight gradient dW[K, N] = dY^T X on a second stream, as in the step
            ws = torch.empty(max(1, m.gemm_tn_ws_floats(0, M, K, N)), device=dev)
            dw = torch.empty(K, N, device=dev)
            tkw = {}
            if f32:
                keep += [C.bound_of_value(torch.linalg.vector_norm(a.float(), float("inf"))),
                         C.bound_of_value(torch.linalg.vector_norm(x.float(), float("inf")))]
                tkw = dict(amax_y=keep[-2].data_ptr(), amax_x=keep[-1].data_ptr())

            def tn_call(stream):
                m.gemm_tn(0, stream, M, K, N, a.data_ptr(), K, x.data_ptr(), N, dw.data_ptr(), ws.data_ptr(), 0.0,
                          f32=f32, **tkw)

            ecin = dict(red, cin=cin.data_ptr(), cmask=cmask.data_ptr())
            t_tn = timeit(lambda: tn_call(st))  # alone (timed on the current stream)

            def both():
                s1.wait_stream(s0)
                nt_call(**ecin)
                tn_call(s1.cuda_stream)
                s0.wait_stream(s1)

            t_both = timeit(both)
            row.update(tn_alone_us=round(t_tn, 1), nt_and_tn_us=round(t_both, 1),
                       overlap_saving_us=round(row["bnred_cin_us"] + t_tn - t_both, 1))
            print(json.dumps(row), flush=True)
            del a, b, c, x, cin, mask, cmask, part, keep, ws, dw
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
