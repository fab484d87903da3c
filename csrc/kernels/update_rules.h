// The update rules of mpiT as per-element functors (host + device).
//
// Each functor takes e[] = the operands at one index, in the order documented on it,
// and updates them in registers. ew.h loads/stores only the arrays each rule reads /
// writes. All math is fp32 regardless of the storage dtype of an operand.
//
// Parity with the reference (file:line in /root/reference):
//   ApplyF         K1  p += a*g            asyncsgd/pserver.lua:91, BiCNN/pserver.lua:138,197
//   ApplySumF      K1  p += a*Σg_k         (fused multi-inbox variant, new)
//   RMSPropF       K2  centered RMSProp    BiCNN/pserver.lua:130-136, optim-rmsprop.lua:49-54
//   AdamF          K3  Adam, host lr_t     BiCNN/pserver.lua:147-154 (stepDivAdam),
//                                          optim-adam-single.lua:24-31 (k = t)
//   AdamaxF        K4  Adamax              BiCNN/pserver.lua:163-170, optim-adamax-single.lua:23-31
//   AdagradF       K5  Adagrad             BiCNN/pserver.lua:177-182, optim-adagrad-single.lua:24-26
//   AdadeltaF      K6  Adadelta            BiCNN/pserver.lua:189-193, optim-adadelta-single.lua:23-27
//   NesterovPreF   K7  vt*=mom; w+=vt      asyncsgd/optim-msgd.lua:27-28, optim-eamsgd.lua:32-33
//   NesterovPostF  K8(+K10b,K14)           asyncsgd/optim-msgd.lua:31-39, optim-eamsgd.lua:36-44,70
//   DownpourF      K9(+K14)                asyncsgd/optim-downpour.lua:24,28,34,44,48
//   ElasticF       K10a sug=mva*(w-w~)     asyncsgd/optim-eamsgd.lua:62-64
//   RegClipF       K11 l1/l2 + clamp       BiCNN/bicnn.lua:398-409
//   ScaleF         K14 g*=a                asyncsgd/goot.lua:213
#pragma once
#include "ew.h"
#include <cmath>

namespace mpit {

// e = [p, g, (out)] ; p += a*g ; out = p
template <bool OUT>
struct ApplyF {
  float a;
  MPIT_HD void operator()(float* e) const {
    e[0] = fmaf(a, e[1], e[0]);
    if constexpr (OUT) e[2] = e[0];
  }
};

// e = [p, g_0..g_{NG-1}, (out)] ; p += a*Σ g_k (summed in inbox order) ; out = p
template <int NG, bool OUT>
struct ApplySumF {
  float a;
  MPIT_HD void operator()(float* e) const {
    float s = e[1];
#pragma unroll
    for (int k = 2; k <= NG; ++k) s += e[k];
    e[0] = fmaf(a, s, e[0]);
    if constexpr (OUT) e[NG + 1] = e[0];
  }
};

// e = [p, g, ga, gs, u, (out)]
//   ga = d*ga + (1-d)*g ; gs = d*gs + (1-d)*g^2 ; r = sqrt(gs - ga^2 + eps)
//   u = mom*u - lr*g/r ; if ADD: p += u ; out = p
template <bool ADD, bool OUT>
struct RMSPropF {
  float decay, lr, mom, eps;
  MPIT_HD void operator()(float* e) const {
    const float g = e[1];
    const float ga = decay * e[2] + (1.f - decay) * g;
    const float gs = decay * e[3] + (1.f - decay) * (g * g);
    const float r = sqrtf(gs - ga * ga + eps);
    const float u = mom * e[4] - lr * (g / r);
    e[2] = ga; e[3] = gs; e[4] = u;
    if constexpr (ADD) e[0] += u;
    if constexpr (OUT) e[5] = e[0];
  }
};

// e = [p, g, m, v, (out)] ; m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2 ;
//   p -= lr_t * m / (sqrt(v) + eps)
template <bool OUT>
struct AdamF {
  float b1, b2, eps, lr_t;
  MPIT_HD void operator()(float* e) const {
    const float g = e[1];
    const float m = b1 * e[2] + (1.f - b1) * g;
    const float v = b2 * e[3] + (1.f - b2) * (g * g);
    e[2] = m; e[3] = v;
    e[0] -= lr_t * (m / (sqrtf(v) + eps));
    if constexpr (OUT) e[4] = e[0];
  }
};

// e = [p, g, m, u, (out)] ; m = b1 m + (1-b1) g ; u = max(b2 u, |g| + eps) ; p -= lr_t m/u
template <bool OUT>
struct AdamaxF {
  float b1, b2, eps, lr_t;
  MPIT_HD void operator()(float* e) const {
    const float g = e[1];
    const float m = b1 * e[2] + (1.f - b1) * g;
    const float u = fmaxf(b2 * e[3], fabsf(g) + eps);
    e[2] = m; e[3] = u;
    e[0] -= lr_t * (m / u);
    if constexpr (OUT) e[4] = e[0];
  }
};

// e = [p, g, var, (out)] ; var += g^2 ; p -= clr * g / (sqrt(var) + eps)
template <bool OUT>
struct AdagradF {
  float eps, clr;
  MPIT_HD void operator()(float* e) const {
    const float g = e[1];
    const float var = e[2] + g * g;
    e[2] = var;
    e[0] -= clr * (g / (sqrtf(var) + eps));
    if constexpr (OUT) e[3] = e[0];
  }
};

// e = [p, g, var, acc, (out)] ; var = rho var + (1-rho) g^2 ; std = sqrt(var + eps)
//   d = sqrt(acc + eps)/std * g ; p -= lr d ; acc = rho acc + (1-rho) d^2
template <bool OUT>
struct AdadeltaF {
  float rho, eps, lr;
  MPIT_HD void operator()(float* e) const {
    const float g = e[1];
    const float var = rho * e[2] + (1.f - rho) * (g * g);
    const float sd = sqrtf(var + eps);
    const float d = (sqrtf(e[3] + eps) / sd) * g;
    e[0] -= lr * d;
    e[2] = var;
    e[3] = rho * e[3] + (1.f - rho) * (d * d);
    if constexpr (OUT) e[4] = e[0];
  }
};

// e = [vt, w] ; vt *= mom ; w += vt
struct NesterovPreF {
  float mom;
  MPIT_HD void operator()(float* e) const {
    e[0] *= mom;
    e[1] += e[0];
  }
};

// e = [w, g, vt, sug] ; g' = gscale*g + l2wd*w ; w -= clr*g' (+ sug) ; vt -= clr*g'
template <bool VT, bool SUG>
struct NesterovPostF {
  float gscale, l2wd, clr;
  MPIT_HD void operator()(float* e) const {
    const float g = gscale * e[1] + l2wd * e[0];
    float w = e[0] - clr * g;
    if constexpr (SUG) w -= e[3];
    e[0] = w;
    if constexpr (VT) e[2] -= clr * g;
  }
};

// e = [g, w, acc] ; d = -lr*(gscale*g + l2wd*w)
//   MODE 0: acc = d            (su == 1: the scaled gradient IS the push buffer)
//   MODE 1: acc += d           (su > 1, sync step: accumulate, then push)
//   MODE 2: acc += d ; w += d  (su > 1, local step: accumulate and move locally)
template <int MODE>
struct DownpourF {
  float lr, gscale, l2wd;
  MPIT_HD void operator()(float* e) const {
    // w is not loaded when l2wd == 0 (its register is undefined): never multiply it
    const float d = -lr * (gscale * e[0] + (l2wd != 0.f ? l2wd * e[1] : 0.f));
    if constexpr (MODE == 0) e[2] = d;
    else e[2] += d;
    if constexpr (MODE == 2) e[1] += d;
  }
};

// e = [w, c, sug] ; sug = mva*(w - c)
struct ElasticF {
  float mva;
  MPIT_HD void operator()(float* e) const { e[2] = mva * (e[0] - e[1]); }
};

// e = [g, p] ; g = clamp(gscale*g + l1*sign(p) + l2*p, -clip, clip)  (clip <= 0: no clamp)
struct RegClipF {
  float gscale, l1, l2, clip;
  MPIT_HD void operator()(float* e) const {
    const float p = e[1];
    const float sg = (p > 0.f) ? 1.f : ((p < 0.f) ? -1.f : 0.f);
    float g = gscale * e[0] + l1 * sg + l2 * p;
    if (clip > 0.f) g = fminf(fmaxf(g, -clip), clip);
    e[0] = g;
  }
};

// e = [x] ; x *= a
struct ScaleF {
  float a;
  MPIT_HD void operator()(float* e) const { e[0] *= a; }
};

// e = [dst, src] ; dst = a*src   (copy / cast when a == 1)
struct CopyF {
  float a;
  MPIT_HD void operator()(float* e) const { e[0] = a * e[1]; }
};

// e = [dst] ; dst = v
struct FillF {
  float v;
  MPIT_HD void operator()(float* e) const { e[0] = v; }
};

// e = [y, x] ; y = a*x + b*y   (general axpby, used by averaging / Reduce_local)
struct AxpbyF {
  float a, b;
  MPIT_HD void operator()(float* e) const { e[0] = a * e[1] + b * e[0]; }
};

}  // namespace mpit
