// Dispatch of the fused update rules (update_rules.h) onto the elementwise engine (ew.h).
// One entry point, ew_update(rule, variant, ...), turns runtime (rule, flags, dtype mask)
// into one of the compiled kernel instantiations. dev < 0 runs the same functor on the
// host (CPU parameter servers — the reference's servers are always CPU,
// asyncsgd/mlaunch.lua:69 — and the gloo plumbing configuration).
#include "kernels.h"
#include "update_rules.h"

namespace mpit {

namespace {

template <int NA, uint32_t RD, uint32_t WR, class F, uint32_t... Ms>
void run_masks(uint32_t bf, const Arrays<NA>& a, int64_t n, const F& f, int dev, hipStream_t s) {
  bool done = ((bf == Ms ? (run_ew<NA, RD, WR, Ms>(a, n, f, dev, s), true) : false) || ...);
  if (!done) throw std::invalid_argument("mpit: unsupported bf16 operand combination for this rule");
}

template <int NA>
Arrays<NA> mk(const std::vector<uintptr_t>& p) {
  if (p.size() != size_t(NA)) throw std::invalid_argument("mpit: wrong number of operands");
  Arrays<NA> a;
  for (int k = 0; k < NA; ++k) a.p[k] = reinterpret_cast<void*>(p[k]);
  return a;
}

constexpr uint32_t bit(int k) { return 1u << k; }
constexpr uint32_t mask_upto(int n) { return (n >= 32) ? 0xffffffffu : ((1u << n) - 1u); }

// Server rules: operand 0 = p (fp32 master), 1 = g (fp32|bf16), 2..NS-1 = fp32 state,
// optional last = out (fp32|bf16, written with the new p).
template <int NS, uint32_t RD, uint32_t WR, class FOut, class FNoOut>
void server_rule(bool out, const std::vector<uintptr_t>& ptrs, uint32_t bf, int64_t n, const FOut& fo,
                 const FNoOut& fn, int dev, hipStream_t s) {
  if (out) {
    constexpr int NA = NS + 1;
    run_masks<NA, RD, WR | bit(NS), FOut, 0u, bit(1), bit(NS), bit(1) | bit(NS)>(bf, mk<NA>(ptrs), n, fo, dev, s);
  } else {
    run_masks<NS, RD, WR, FNoOut, 0u, bit(1)>(bf, mk<NS>(ptrs), n, fn, dev, s);
  }
}

template <int NG>
void apply_sum(bool out, const std::vector<uintptr_t>& ptrs, uint32_t bf, int64_t n, float a, int dev,
               hipStream_t s) {
  constexpr uint32_t RD = mask_upto(NG + 1);
  if (out) {
    run_masks<NG + 2, RD, bit(0) | bit(NG + 1), ApplySumF<NG, true>, 0u, bit(NG + 1)>(
        bf, mk<NG + 2>(ptrs), n, ApplySumF<NG, true>{a}, dev, s);
  } else {
    run_masks<NG + 1, RD, bit(0), ApplySumF<NG, false>, 0u>(bf, mk<NG + 1>(ptrs), n, ApplySumF<NG, false>{a},
                                                            dev, s);
  }
}

float S(const std::vector<float>& sc, size_t i) {
  if (i >= sc.size()) throw std::invalid_argument("mpit: missing scalar argument");
  return sc[i];
}

}  // namespace

void ew_update(int rule, int variant, int dev, hipStream_t s, int64_t n, const std::vector<uintptr_t>& ptrs,
               uint32_t bf, const std::vector<float>& sc) {
  if (dev >= 0) hip_check(hipSetDevice(dev), "hipSetDevice");
  const bool out = (variant & kOut) != 0;
  switch (rule) {
    case kApply:
      server_rule<2, bit(0) | bit(1), bit(0)>(out, ptrs, bf, n, ApplyF<true>{S(sc, 0)}, ApplyF<false>{S(sc, 0)},
                                             dev, s);
      break;
    case kApplySum: {
      const int ng = variant >> 8;
      const float a = S(sc, 0);
      switch (ng) {
        case 1: server_rule<2, bit(0) | bit(1), bit(0)>(out, ptrs, bf, n, ApplyF<true>{a}, ApplyF<false>{a}, dev, s); break;
        case 2: apply_sum<2>(out, ptrs, bf, n, a, dev, s); break;
        case 3: apply_sum<3>(out, ptrs, bf, n, a, dev, s); break;
        case 4: apply_sum<4>(out, ptrs, bf, n, a, dev, s); break;
        case 5: apply_sum<5>(out, ptrs, bf, n, a, dev, s); break;
        case 6: apply_sum<6>(out, ptrs, bf, n, a, dev, s); break;
        case 7: apply_sum<7>(out, ptrs, bf, n, a, dev, s); break;
        case 8: apply_sum<8>(out, ptrs, bf, n, a, dev, s); break;
        default: throw std::invalid_argument("mpit: apply_sum supports 1..8 gradient inboxes");
      }
      break;
    }
    case kRMSProp: {
      const float d = S(sc, 0), lr = S(sc, 1), mom = S(sc, 2), eps = S(sc, 3);
      constexpr uint32_t RD = bit(0) | bit(1) | bit(2) | bit(3) | bit(4);
      if (variant & kAdd) {
        server_rule<5, RD, bit(0) | bit(2) | bit(3) | bit(4)>(out, ptrs, bf, n, RMSPropF<true, true>{d, lr, mom, eps},
                                                             RMSPropF<true, false>{d, lr, mom, eps}, dev, s);
      } else {
        // local mode: only the state and the update u are produced (p operand unused)
        constexpr uint32_t RDn = bit(1) | bit(2) | bit(3) | bit(4);
        run_masks<5, RDn, bit(2) | bit(3) | bit(4), RMSPropF<false, false>, 0u, bit(1)>(
            bf, mk<5>(ptrs), n, RMSPropF<false, false>{d, lr, mom, eps}, dev, s);
      }
      break;
    }
    case kAdam: {
      AdamF<true> fo{S(sc, 0), S(sc, 1), S(sc, 2), S(sc, 3)};
      AdamF<false> fn{S(sc, 0), S(sc, 1), S(sc, 2), S(sc, 3)};
      server_rule<4, bit(0) | bit(1) | bit(2) | bit(3), bit(0) | bit(2) | bit(3)>(out, ptrs, bf, n, fo, fn, dev, s);
      break;
    }
    case kAdamax: {
      AdamaxF<true> fo{S(sc, 0), S(sc, 1), S(sc, 2), S(sc, 3)};
      AdamaxF<false> fn{S(sc, 0), S(sc, 1), S(sc, 2), S(sc, 3)};
      server_rule<4, bit(0) | bit(1) | bit(2) | bit(3), bit(0) | bit(2) | bit(3)>(out, ptrs, bf, n, fo, fn, dev, s);
      break;
    }
    case kAdagrad: {
      AdagradF<true> fo{S(sc, 0), S(sc, 1)};
      AdagradF<false> fn{S(sc, 0), S(sc, 1)};
      server_rule<3, bit(0) | bit(1) | bit(2), bit(0) | bit(2)>(out, ptrs, bf, n, fo, fn, dev, s);
      break;
    }
    case kAdadelta: {
      AdadeltaF<true> fo{S(sc, 0), S(sc, 1), S(sc, 2)};
      AdadeltaF<false> fn{S(sc, 0), S(sc, 1), S(sc, 2)};
      server_rule<4, bit(0) | bit(1) | bit(2) | bit(3), bit(0) | bit(2) | bit(3)>(out, ptrs, bf, n, fo, fn, dev, s);
      break;
    }
    case kNesterovPre:
      run_masks<2, bit(0) | bit(1), bit(0) | bit(1), NesterovPreF, 0u>(bf, mk<2>(ptrs), n, NesterovPreF{S(sc, 0)},
                                                                        dev, s);
      break;
    case kNesterovPost: {
      const float gs = S(sc, 0), l2 = S(sc, 1), clr = S(sc, 2);
      const bool vt = variant & kVt, sug = variant & kSug;
      // operands always [w, g, vt, sug]; unused ones are neither read nor written
      if (vt && sug)
        run_masks<4, 0xfu, bit(0) | bit(2), NesterovPostF<true, true>, 0u, bit(1), bit(3), bit(1) | bit(3)>(
            bf, mk<4>(ptrs), n, NesterovPostF<true, true>{gs, l2, clr}, dev, s);
      else if (vt)
        run_masks<4, 0x7u, bit(0) | bit(2), NesterovPostF<true, false>, 0u, bit(1)>(
            bf, mk<4>(ptrs), n, NesterovPostF<true, false>{gs, l2, clr}, dev, s);
      else if (sug)
        run_masks<4, bit(0) | bit(1) | bit(3), bit(0), NesterovPostF<false, true>, 0u, bit(1), bit(3), bit(1) | bit(3)>(
            bf, mk<4>(ptrs), n, NesterovPostF<false, true>{gs, l2, clr}, dev, s);
      else
        run_masks<4, 0x3u, bit(0), NesterovPostF<false, false>, 0u, bit(1)>(
            bf, mk<4>(ptrs), n, NesterovPostF<false, false>{gs, l2, clr}, dev, s);
      break;
    }
    case kDownpour: {
      const float lr = S(sc, 0), gs = S(sc, 1), l2 = S(sc, 2);
      const int mode = variant & 3;
      const bool rw = (l2 != 0.f);  // w is only read for weight decay (or written in mode 2)
      if (mode == 0) {
        if (rw)
          run_masks<3, bit(0) | bit(1), bit(2), DownpourF<0>, 0u, bit(0), bit(2), bit(0) | bit(2)>(
              bf, mk<3>(ptrs), n, DownpourF<0>{lr, gs, l2}, dev, s);
        else
          run_masks<3, bit(0), bit(2), DownpourF<0>, 0u, bit(0), bit(2), bit(0) | bit(2)>(
              bf, mk<3>(ptrs), n, DownpourF<0>{lr, gs, 0.f}, dev, s);
      } else if (mode == 1) {
        if (rw)
          run_masks<3, 0x7u, bit(2), DownpourF<1>, 0u, bit(0)>(bf, mk<3>(ptrs), n, DownpourF<1>{lr, gs, l2}, dev, s);
        else
          run_masks<3, bit(0) | bit(2), bit(2), DownpourF<1>, 0u, bit(0)>(bf, mk<3>(ptrs), n,
                                                                           DownpourF<1>{lr, gs, 0.f}, dev, s);
      } else {
        run_masks<3, 0x7u, bit(1) | bit(2), DownpourF<2>, 0u, bit(0)>(bf, mk<3>(ptrs), n, DownpourF<2>{lr, gs, l2},
                                                                       dev, s);
      }
      break;
    }
    case kElastic:
      run_masks<3, bit(0) | bit(1), bit(2), ElasticF, 0u, bit(2)>(bf, mk<3>(ptrs), n, ElasticF{S(sc, 0)}, dev, s);
      break;
    case kRegClip:
      run_masks<2, 0x3u, bit(0), RegClipF, 0u, bit(0)>(bf, mk<2>(ptrs), n,
                                                       RegClipF{S(sc, 0), S(sc, 1), S(sc, 2), S(sc, 3)}, dev, s);
      break;
    case kScale:
      run_masks<1, 1u, 1u, ScaleF, 0u, 1u>(bf, mk<1>(ptrs), n, ScaleF{S(sc, 0)}, dev, s);
      break;
    case kCopy:
      run_masks<2, bit(1), bit(0), CopyF, 0u, 1u, 2u, 3u>(bf, mk<2>(ptrs), n, CopyF{S(sc, 0)}, dev, s);
      break;
    case kFill:
      run_masks<1, 0u, 1u, FillF, 0u, 1u>(bf, mk<1>(ptrs), n, FillF{S(sc, 0)}, dev, s);
      break;
    case kAxpby:
      run_masks<2, 0x3u, bit(0), AxpbyF, 0u, 1u, 2u, 3u>(bf, mk<2>(ptrs), n, AxpbyF{S(sc, 0), S(sc, 1)}, dev, s);
      break;
    default:
      throw std::invalid_argument("mpit: unknown update rule " + std::to_string(rule));
  }
}

void ew_update_multi(int rule, int variant, int dev, hipStream_t s, const std::vector<int64_t>& ns,
                     const std::vector<std::vector<uintptr_t>>& ptrs, uint32_t bf, const std::vector<float>& sc) {
  if (ns.size() != ptrs.size()) throw std::invalid_argument("mpit: ew_update_multi: one operand list per segment");
  if (ns.empty()) return;
  if (ns.size() == 1) {
    ew_update(rule, variant, dev, s, ns[0], ptrs[0], bf, sc);
    return;
  }
  const MultiSegs ms{ptrs, ns};
  struct Reset {
    ~Reset() { t_multi = nullptr; }
  } reset;
  t_multi = &ms;  // consumed by the one run_ew the rule dispatch reaches
  ew_update(rule, variant, dev, s, ns[0], ptrs[0], bf, sc);
}

}  // namespace mpit
