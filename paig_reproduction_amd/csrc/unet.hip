// The whole U-Net, forward and backward, as one C-ABI call each way
// (paig_unet_fwd / paig_unet_bwd): ShallowUNet
// (nn/network/blocks.py:240-308) or UNet (:106-237) over F frames.
//
// This is the plan interpreter of the Python engine (engine.py:
// shallow_unet_plan, unet_plan, backward_plan, Engine._unet_forward,
// Engine._unet_backward) restated in C++ over the library's own entry
// points, so a host without this package's Python runs the U-Net through the
// C ABI alone.  The same kernels run in the same order with the same
// arguments (fused pools / upsamples, weight images, max-|x| slots, fused
// layer backwards, one batched slab reduction), so the results are
// bit-identical to the Python engine's (tests/test_gpu_unet_abi.py) in its
// default configuration (the engine's A/B switches map to the _ex flags:
// PAIG_FUSED_BWD=0 -> PAIG_UNET_SEPARATE_BWD, PAIG_UPT=0 ->
// PAIG_UNET_STANDALONE_UP, PAIG_POOL_FOLD=0 -> PAIG_UNET_STANDALONE_POOL).
// Host code only; the caller's workspace holds every activation, gradient
// and partial-gradient slab (paig_unet_workspace), the library allocates
// nothing.
#include "common.h"

#include <vector>

#define UNET_HIP(call)                                                  \
  do {                                                                  \
    const hipError_t _e = (call);                                       \
    if (_e != hipSuccess) {                                             \
      paig_set_error("%s: %s", __func__, hipGetErrorString(_e));        \
      return (int)_e;                                                   \
    }                                                                   \
  } while (0)

namespace {

enum { U_CONV = 0, U_POOL = 1, U_UP = 2 };

struct Reg {
  int buf, off, n;
  bool operator==(const Reg& o) const { return buf == o.buf && off == o.off && n == o.n; }
};
struct UOp {
  int kind;
  int conv;   // index among the convs (parameter order), -1 for pool / up
  Reg src, dst;
  bool relu;
  int ks;
};
struct UBuf {
  int C, lvl;
};

struct UPlan {
  std::vector<UBuf> bufs;
  std::vector<UOp> ops;
  int nconv = 0, X0 = 0, LG = 0;
  // derived: per op the regions it finalizes (earliest consumer of a
  // producer's output) with their ReLU; per conv op the fused upsample op
  // (-1: none); per buffer: an upsampled tensor formed inside its consumer
  std::vector<std::vector<std::pair<Reg, bool>>> fin;
  std::vector<int> fused_up;
  std::vector<bool> fused_buf;
};

// engine.py shallow_unet_plan (c = 8) / unet_plan (h = 16)
void build_plan(UPlan& p, int net, int K) {
  auto buf = [&](int C, int lvl) {
    p.bufs.push_back(UBuf{C, lvl});
    return (int)p.bufs.size() - 1;
  };
  auto conv = [&](Reg s, Reg d, bool relu, int ks = 3) { p.ops.push_back(UOp{U_CONV, p.nconv++, s, d, relu, ks}); };
  auto pool = [&](Reg s, Reg d) { p.ops.push_back(UOp{U_POOL, -1, s, d, false, 0}); };
  auto up = [&](Reg s, Reg d) { p.ops.push_back(UOp{U_UP, -1, s, d, false, 0}); };
  if (net == 0) {
    const int c = 8;
    const int X0 = buf(3, 1), A1 = buf(c, 1), CAT2 = buf(3 * c, 1), P1 = buf(c, 2), A3 = buf(2 * c, 2),
              CAT1 = buf(4 * c, 2), P2 = buf(2 * c, 4), A5 = buf(4 * c, 4), A6 = buf(4 * c, 4), U1 = buf(4 * c, 2),
              A8 = buf(2 * c, 2), A9 = buf(2 * c, 2), U2 = buf(2 * c, 1), A11 = buf(c, 1), A12 = buf(c, 1),
              LG = buf(K, 1);
    p.X0 = X0;
    p.LG = LG;
    conv({X0, 0, 3}, {A1, 0, c}, true);
    conv({A1, 0, c}, {CAT2, 2 * c, c}, true);
    pool({CAT2, 2 * c, c}, {P1, 0, c});
    conv({P1, 0, c}, {A3, 0, 2 * c}, true);
    conv({A3, 0, 2 * c}, {CAT1, 2 * c, 2 * c}, true);
    pool({CAT1, 2 * c, 2 * c}, {P2, 0, 2 * c});
    conv({P2, 0, 2 * c}, {A5, 0, 4 * c}, true);
    conv({A5, 0, 4 * c}, {A6, 0, 4 * c}, true);
    up({A6, 0, 4 * c}, {U1, 0, 4 * c});
    conv({U1, 0, 4 * c}, {CAT1, 0, 2 * c}, false);
    conv({CAT1, 0, 4 * c}, {A8, 0, 2 * c}, true);
    conv({A8, 0, 2 * c}, {A9, 0, 2 * c}, true);
    up({A9, 0, 2 * c}, {U2, 0, 2 * c});
    conv({U2, 0, 2 * c}, {CAT2, 0, 2 * c}, false);
    conv({CAT2, 0, 3 * c}, {A11, 0, c}, true);
    conv({A11, 0, c}, {A12, 0, c}, true);
    conv({A12, 0, c}, {LG, 0, K}, true, 1);   // c13, ReLU'd (Q13)
  } else {
    const int h = 16;
    const int X0 = buf(3, 1), A1 = buf(h, 1), CAT3 = buf(3 * h, 1), P1 = buf(h, 2), A3 = buf(2 * h, 2),
              CAT2 = buf(4 * h, 2), P2 = buf(2 * h, 4), A5 = buf(4 * h, 4), CAT1 = buf(6 * h, 4), P3 = buf(4 * h, 8),
              A7 = buf(8 * h, 8), A8 = buf(8 * h, 8), U1 = buf(8 * h, 4), A10 = buf(4 * h, 4), A11 = buf(4 * h, 4),
              U2 = buf(4 * h, 2), A13 = buf(2 * h, 2), A14 = buf(2 * h, 2), U3 = buf(2 * h, 1), A16 = buf(h, 1),
              A17 = buf(h, 1), LG = buf(K, 1);
    p.X0 = X0;
    p.LG = LG;
    conv({X0, 0, 3}, {A1, 0, h}, true);
    conv({A1, 0, h}, {CAT3, 2 * h, h}, true);
    pool({CAT3, 2 * h, h}, {P1, 0, h});
    conv({P1, 0, h}, {A3, 0, 2 * h}, true);
    conv({A3, 0, 2 * h}, {CAT2, 2 * h, 2 * h}, true);
    pool({CAT2, 2 * h, 2 * h}, {P2, 0, 2 * h});
    conv({P2, 0, 2 * h}, {A5, 0, 4 * h}, true);
    conv({A5, 0, 4 * h}, {CAT1, 2 * h, 4 * h}, true);
    pool({CAT1, 2 * h, 4 * h}, {P3, 0, 4 * h});
    conv({P3, 0, 4 * h}, {A7, 0, 8 * h}, true);
    conv({A7, 0, 8 * h}, {A8, 0, 8 * h}, true);
    up({A8, 0, 8 * h}, {U1, 0, 8 * h});
    conv({U1, 0, 8 * h}, {CAT1, 0, 2 * h}, false);
    conv({CAT1, 0, 6 * h}, {A10, 0, 4 * h}, true);
    conv({A10, 0, 4 * h}, {A11, 0, 4 * h}, true);
    up({A11, 0, 4 * h}, {U2, 0, 4 * h});
    conv({U2, 0, 4 * h}, {CAT2, 0, 2 * h}, false);
    conv({CAT2, 0, 4 * h}, {A13, 0, 2 * h}, true);
    conv({A13, 0, 2 * h}, {A14, 0, 2 * h}, true);
    up({A14, 0, 2 * h}, {U3, 0, 2 * h});
    conv({U3, 0, 2 * h}, {CAT3, 0, 2 * h}, false);
    conv({CAT3, 0, 3 * h}, {A16, 0, h}, true);
    conv({A16, 0, h}, {A17, 0, h}, true);
    conv({A17, 0, h}, {LG, 0, K}, false, 1);   // c18, not ReLU'd
  }
}

bool overlap(const Reg& a, const Reg& b) { return a.buf == b.buf && a.off < b.off + b.n && b.off < a.off + a.n; }

// engine.py backward_plan and Layout's fused upsamples
void derive(UPlan& p, int H, int cm) {
  const int n = (int)p.ops.size();
  p.fin.assign(n, {});
  for (int pi = 0; pi < n; ++pi) {
    int first = -1;
    for (int i = pi + 1; i < n && first < 0; ++i)
      if (overlap(p.ops[i].src, p.ops[pi].dst)) first = i;
    if (first >= 0) p.fin[first].push_back({p.ops[pi].dst, p.ops[pi].kind == U_CONV && p.ops[pi].relu});
  }
  p.fused_up.assign(n, -1);
  p.fused_buf.assign(p.bufs.size(), false);
  for (int i = 0; i < n; ++i) {
    const UOp& u = p.ops[i];
    if (u.kind != U_UP) continue;
    int cons = -1, ncons = 0;
    for (int j = 0; j < n; ++j)
      if (p.ops[j].src.buf == u.dst.buf) {
        cons = j;
        ++ncons;
      }
    if (ncons != 1 || p.ops[cons].kind != U_CONV) continue;
    const UOp& c = p.ops[cons];
    const int Hc = H / p.bufs[u.dst.buf].lvl;
    bool ok = true;
    for (int w = 0; w < 2; ++w)
      ok = ok && paig_conv2d_mfma_supported(w, c.src.n, c.dst.n, Hc, Hc, c.ks, 32 | cm);
    if (ok) {
      p.fused_up[cons] = i;
      p.fused_buf[u.dst.buf] = true;
    }
  }
}

// the conv op i's 2x2 pool (next op) is fused into its forward epilogue /
// folded into its layer backward
bool pool_fused(const UPlan& p, int i, int H, int cm) {
  const UOp& op = p.ops[i];
  if (op.kind != U_CONV || i + 1 >= (int)p.ops.size() || cm == 0 || p.fused_up[i] >= 0) return false;
  const UOp& nx = p.ops[i + 1];
  const int Hl = H / p.bufs[op.dst.buf].lvl;
  return nx.kind == U_POOL && nx.src == op.dst &&
         paig_conv2d_mfma_supported(0, op.src.n, op.dst.n, Hl, Hl, op.ks, cm | 64);
}
// the pool's backward folded into the fused layer backward's dY staging, or
// (layers too wide for it: the UNet's c4) into the separate weight gradient's
// and data gradient's staging (paig_conv2d_wgrad_pf, paig_conv2d_fwd_pwc
// flags 8 | 64)
bool pool_fold_fused(const UPlan& p, int i, int H, int cm) {
  const UOp& op = p.ops[i];
  const int Hl = H / p.bufs[op.dst.buf].lvl;
  return paig_conv2d_bwd_supported(op.src.n, op.dst.n, Hl, Hl, op.ks, cm | 64);
}
bool pool_fold_split(const UPlan& p, int i, int H, int cm, int flags) {
  const UOp& op = p.ops[i];
  const int Hl = H / p.bufs[op.dst.buf].lvl;
  // (not for a layer that takes the fused layer backward without a pool
  // instantiation: that launch would get the codes and flag 64 it cannot fold)
  return cm == 128 && !(flags & PAIG_UNET_STANDALONE_POOL) && op.src.buf != p.X0 && !pool_fold_fused(p, i, H, cm) &&
         !paig_conv2d_bwd_supported(op.src.n, op.dst.n, Hl, Hl, op.ks, cm) &&
         paig_conv2d_mfma_supported(1, op.src.n, op.dst.n, Hl, Hl, op.ks, 128 | 64) &&
         paig_conv2d_mfma_supported(0, op.dst.n, op.src.n, Hl, Hl, op.ks, 8 | 128 | 64);
}
// (the codes come from the fused pool, or from the standalone pool where the
// forward cannot fuse it: paig_maxpool2_fwd_codes)
bool pool_folded(const UPlan& p, int i, int H, int cm, int flags) {
  const UOp& op = p.ops[i];
  if (flags & (PAIG_UNET_SEPARATE_BWD | PAIG_UNET_INFERENCE)) return false;
  if (op.kind != U_CONV || i + 1 >= (int)p.ops.size() || cm == 0 || p.fused_up[i] >= 0) return false;
  const UOp& nx = p.ops[i + 1];
  const int Hl = H / p.bufs[op.dst.buf].lvl;
  return nx.kind == U_POOL && nx.src == op.dst && (pool_fold_fused(p, i, H, cm) || pool_fold_split(p, i, H, cm, flags));
}

constexpr int NBLK_MAX = 1024;   // slab rows per conv (engine.py: nblk_max)
size_t a256(size_t b) { return (b + 255) & ~(size_t)255; }

// Workspace layout (bytes), shared by the query and both calls
struct ULayout {
  std::vector<size_t> act, grad, slab, wprep0, wprep1, pcode;   // offsets (SIZE_MAX: none)
  std::vector<long long> pcode_fs;
  size_t xmax = 0, total = 0;
};

// flags: PAIG_UNET_INFERENCE -> no gradient buffers, slabs or pool codes;
// PAIG_UNET_EXT_WPREP -> no weight images (the caller's)
void layout(const UPlan& p, ULayout& L, int F, int H, int cm, int flags) {
  const bool train = !(flags & PAIG_UNET_INFERENCE);
  const size_t NONE = (size_t)-1;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += a256(bytes);
    return o;
  };
  const int nb = (int)p.bufs.size(), no = (int)p.ops.size();
  L.act.assign(nb, NONE);
  L.grad.assign(nb, NONE);
  for (int b = 0; b < nb; ++b) {
    const size_t hw = (size_t)(H / p.bufs[b].lvl) * (H / p.bufs[b].lvl);
    const size_t bytes = (size_t)F * p.bufs[b].C * hw * 4;
    if (b != p.X0 && b != p.LG && !p.fused_buf[b]) L.act[b] = take(bytes);
    if (b != p.X0 && train) L.grad[b] = take(bytes);
  }
  L.xmax = take((size_t)no * PAIG_XMAX_SLOTS * 4);
  L.slab.assign(no, NONE);
  L.wprep0.assign(no, NONE);
  L.wprep1.assign(no, NONE);
  L.pcode.assign(no, NONE);
  L.pcode_fs.assign(no, 0);
  for (int i = 0; i < no; ++i) {
    const UOp& op = p.ops[i];
    if (op.kind != U_CONV) continue;
    const int cin = op.src.n, cout = op.dst.n, ks = op.ks;
    if (train) L.slab[i] = take((size_t)NBLK_MAX * (cout * cin * ks * ks + cout) * 4);
    if (cm == 128 && !(flags & PAIG_UNET_EXT_WPREP)) {
      L.wprep0[i] = take((size_t)paig_conv_wprep_size(cin, cout, ks) * 2);
      if (op.src.buf != p.X0) L.wprep1[i] = take((size_t)paig_conv_wprep_size(cout, cin, ks) * 2);
    }
    if (pool_folded(p, i, H, cm, flags)) {
      const int Hl = H / p.bufs[op.dst.buf].lvl;
      L.pcode_fs[i + 1] = (long long)((cout + 7) / 8 * 8) * (Hl / 2) * (Hl / 2);
      L.pcode[i + 1] = take((size_t)F * L.pcode_fs[i + 1]);
    }
  }
  L.total = off;
}

struct View {
  const float* p;
  long long fs;
  int grp;
  long long gs;
};

int check_args(int net, int F, int H, int K, int cm) {
  PAIG_REQUIRE(net == 0 || net == 1, "paig_unet: net %d (0 ShallowUNet, 1 UNet)", net);
  PAIG_REQUIRE(F > 0 && H > 0 && H % (net == 0 ? 4 : 8) == 0 && K > 0, "paig_unet: F=%d H=%d K=%d", F, H, K);
  PAIG_REQUIRE(cm == 0 || cm == 128 || cm == 256, "paig_unet: conv math %d (0 fp32, 128 split, 256 bf16)", cm);
  return 0;
}

// per-launch probe (the engine's HIP-event timing of one conv launch;
// bench.py's roofline): event 0 before, 1 after the launch
struct UProbe {
  paig_unet_probe_fn fn;
  void* ctx;
  void operator()(int ev, int op, int conv, int kind, int cin, int cout, int Hl, int fl) const {
    if (fn) fn(ctx, ev, op, conv, kind, cin, cout, Hl, fl);
  }
};

int fwd_impl(int net, int F, int H, int K, int math, int flags, const float* x, long long x_fs, int x_grp,
             long long x_gs, const float* const* w, const float* const* b, float* logits, const void* const* wpf,
             const void* const* wpd, void* ws, size_t ws_bytes, UProbe pr, void* stream) {
  // weight prep deferred by the caller (paig_conv_wprep_defer): the first
  // split forward takes it; whatever is left runs before this call returns
  struct WprepFlush {
    void* st;
    ~WprepFlush() { (void)paig_conv_wprep_flush(st); }
  } wflush{stream};
  if (int rc = check_args(net, F, H, K, math)) return rc;
  UPlan p;
  build_plan(p, net, K);
  derive(p, H, math);
  ULayout L;
  layout(p, L, F, H, math, flags);
  const bool head = (flags & PAIG_UNET_HEAD_FUSED) != 0, ext = (flags & PAIG_UNET_EXT_WPREP) != 0;
  PAIG_REQUIRE(ws && ws_bytes >= L.total && x && (logits || head) && w && b && (!ext || math != 128 || (wpf && wpd)),
               "paig_unet_fwd: workspace %zu bytes < %zu, or a null operand", ws_bytes, L.total);
  char* base = static_cast<char*>(ws);
  const int cm = math;
  auto view = [&](const Reg& r, int& lvl) {
    lvl = p.bufs[r.buf].lvl;
    const long long hw = (long long)(H / lvl) * (H / lvl);
    if (r.buf == p.X0) return View{x + r.off * hw, x_fs, x_grp, x_gs};
    float* t = r.buf == p.LG ? logits : reinterpret_cast<float*>(base + L.act[r.buf]);
    return View{t + r.off * hw, p.bufs[r.buf].C * hw, 0, 0};
  };
  // the per-block max |x| slots (the split forward writes its layer's; a slot
  // no forward wrote must read zero: the wgrad then takes the guarded fixed
  // scale instead of a garbage exponent)
  // (the first layer's split forward zeroes the others' slots: no memset on
  // the step's critical path; a memset of all of them when it did not)
  float* xmax = reinterpret_cast<float*>(base + L.xmax);
  const size_t xmax_n = p.ops.size() * PAIG_XMAX_SLOTS;
  static const bool memset_ab = getenv("PAIG_XMAX_MEMSET") != nullptr;   // A/B: the round-5 memset
  const bool prezero =
      !memset_ab && !p.ops.empty() && p.ops[0].kind == U_CONV && p.fused_up[0] < 0 && p.ops.size() > 1;
  if (prezero) paig_conv_fwd_prezero(xmax + PAIG_XMAX_SLOTS, (int)(xmax_n - PAIG_XMAX_SLOTS));
  else UNET_HIP(hipMemsetAsync(xmax, 0, xmax_n * 4, (hipStream_t)stream));
  const int no = (int)p.ops.size(), nrun = head ? no - 1 : no;   // HEAD_FUSED: the 1x1 head is the caller's
  auto wimg0 = [&](int i) -> const void* {
    return cm != 128 ? nullptr : (ext ? wpf[p.ops[i].conv] : base + L.wprep0[i]);
  };
  if (cm == 128 && !ext) {   // every conv's forward / dgrad weight images, one launch
    std::vector<const float*> jw;
    std::vector<int> jci, jco, jks, jdg;
    std::vector<void*> jout;
    for (int i = 0; i < no; ++i) {
      const UOp& op = p.ops[i];
      if (op.kind != U_CONV) continue;
      jw.push_back(w[op.conv]), jci.push_back(op.src.n), jco.push_back(op.dst.n), jks.push_back(op.ks),
          jdg.push_back(0), jout.push_back(base + L.wprep0[i]);
      if (op.src.buf != p.X0)
        jw.push_back(w[op.conv]), jci.push_back(op.dst.n), jco.push_back(op.src.n), jks.push_back(op.ks),
            jdg.push_back(1), jout.push_back(base + L.wprep1[i]);
    }
    if (int rc = paig_conv_wprep((int)jw.size(), jw.data(), jci.data(), jco.data(), jks.data(), jdg.data(),
                                 jout.data(), stream))
      return rc;
  }
  std::vector<bool> pooled(no, false);
  for (int i = 0; i < nrun; ++i) {
    const UOp& op = p.ops[i];
    if ((op.kind == U_UP && p.fused_buf[op.dst.buf]) || pooled[i]) continue;
    int dlvl;
    const View dv = view(op.dst, dlvl);
    int rc = 0;
    if (op.kind == U_CONV) {
      int slvl, xfl = 0;
      View sv;
      if (p.fused_up[i] >= 0) {
        sv = view(p.ops[p.fused_up[i]].src, slvl);
        slvl /= 2;
        xfl = 32;
      } else {
        sv = view(op.src, slvl);
      }
      const int Hl = H / slvl;
      float* pool_out = nullptr;
      long long pool_fs = 0;
      unsigned char* pcode = nullptr;
      long long pcode_fs = 0;
      if (pool_fused(p, i, H, cm) && i + 1 < nrun) {
        int pl;
        const View pv = view(p.ops[i + 1].dst, pl);
        pool_out = const_cast<float*>(pv.p);
        pool_fs = pv.fs;
        pooled[i + 1] = true;
        if (L.pcode[i + 1] != (size_t)-1) {
          pcode = reinterpret_cast<unsigned char*>(base + L.pcode[i + 1]);
          pcode_fs = L.pcode_fs[i + 1];
        }
      }
      const int fl = (op.relu ? 1 : 0) | xfl | cm | (pool_out ? 64 : 0);
      pr(0, i, op.conv, PAIG_PROBE_CONV_FWD, op.src.n, op.dst.n, Hl, fl);
      rc = paig_conv2d_fwd_pwc(sv.p, sv.fs, sv.grp, sv.gs, const_cast<float*>(dv.p), dv.fs, nullptr, 0, w[op.conv],
                               b[op.conv], F, op.src.n, op.dst.n, Hl, Hl, op.ks, fl,
                               xmax + (size_t)i * PAIG_XMAX_SLOTS, PAIG_XMAX_SLOTS, pool_out, pool_fs, pcode, pcode_fs,
                               wimg0(i), stream);
      pr(1, i, op.conv, PAIG_PROBE_CONV_FWD, op.src.n, op.dst.n, Hl, fl);
      if (i == 0 && prezero && paig_conv_fwd_prezero_pending()) {
        if (rc) return rc;
        UNET_HIP(hipMemsetAsync(xmax, 0, xmax_n * 4, (hipStream_t)stream));   // no split forward took the range
      }
    } else if (op.kind == U_POOL) {
      int slvl;
      const View sv = view(op.src, slvl);
      const int Hl = H / slvl;
      rc = L.pcode[i] != (size_t)-1
               ? paig_maxpool2_fwd_codes(sv.p, sv.fs, const_cast<float*>(dv.p), dv.fs,
                                         reinterpret_cast<unsigned char*>(base + L.pcode[i]), L.pcode_fs[i], F,
                                         op.src.n, Hl, Hl, stream)
               : paig_maxpool2_fwd(sv.p, sv.fs, const_cast<float*>(dv.p), dv.fs, F, op.src.n, Hl, Hl, stream);
    } else {
      int slvl;
      const View sv = view(op.src, slvl);
      const int Hs = H / slvl, Ho = H / dlvl;
      rc = paig_upsample2_fwd(sv.p, sv.fs, const_cast<float*>(dv.p), dv.fs, F, op.src.n, Hs, Hs, Ho, Ho, stream);
    }
    if (rc) return rc;
  }
  return 0;
}

int bwd_impl(int net, int F, int H, int K, int math, int flags, const float* x, long long x_fs, int x_grp,
             long long x_gs, const float* const* w, const float* logits, const float* dlogits, float* const* dwb,
             int n_extra, const float* const* e_src, const int* e_nb, const int* e_len, float* const* e_dst,
             const void* const* wpd, void* ws, size_t ws_bytes, UProbe pr, void* stream) {
  if (int rc = check_args(net, F, H, K, math)) return rc;
  UPlan p;
  build_plan(p, net, K);
  derive(p, H, math);
  ULayout L;
  layout(p, L, F, H, math, flags);
  const bool head = (flags & PAIG_UNET_HEAD_FUSED) != 0, ext = (flags & PAIG_UNET_EXT_WPREP) != 0;
  const bool sep = (flags & PAIG_UNET_SEPARATE_BWD) != 0;
  PAIG_REQUIRE(!(flags & PAIG_UNET_INFERENCE), "paig_unet_bwd: the forward ran in inference mode (no gradients)");
  PAIG_REQUIRE(ws && ws_bytes >= L.total && x && (head || (logits && dlogits)) && w && dwb &&
                   (!ext || math != 128 || wpd) && n_extra >= 0 && (n_extra == 0 || (e_src && e_nb && e_len && e_dst)),
               "paig_unet_bwd: workspace %zu bytes < %zu, or a null operand", ws_bytes, L.total);
  char* base = static_cast<char*>(ws);
  hipStream_t st = (hipStream_t)stream;
  const int cm = math, no = (int)p.ops.size();
  float* xmax = reinterpret_cast<float*>(base + L.xmax);
  auto view = [&](const Reg& r, int& lvl) {
    lvl = p.bufs[r.buf].lvl;
    const long long hw = (long long)(H / lvl) * (H / lvl);
    if (r.buf == p.X0) return View{x + r.off * hw, x_fs, x_grp, x_gs};
    const float* t = r.buf == p.LG ? logits : reinterpret_cast<const float*>(base + L.act[r.buf]);
    return View{t + r.off * hw, p.bufs[r.buf].C * hw, 0, 0};
  };
  auto dview = [&](const Reg& r) {
    const long long hw = (long long)(H / p.bufs[r.buf].lvl) * (H / p.bufs[r.buf].lvl);
    float* t = reinterpret_cast<float*>(base + L.grad[r.buf]);
    return View{t + r.off * hw, p.bufs[r.buf].C * hw, 0, 0};
  };
  // write / accumulate state of every gradient region (engine.py state/mark)
  std::vector<std::vector<std::pair<int, int>>> written(p.bufs.size());
  int first;
  if (head) {
    // the caller's fused head backward wrote the head input's gradient (its
    // producer's ReLU' applied) into the workspace (paig_unet_buffer)
    const Reg hs = p.ops[no - 1].src;
    written[hs.buf].push_back({hs.off, hs.n});
    first = no - 2;
  } else {
    // d logits: the caller's gradient, with ShallowUNet c13's ReLU' (Q13)
    float* dlg = reinterpret_cast<float*>(base + L.grad[p.LG]);
    const long long nlg = (long long)F * K * H * H;
    UNET_HIP(hipMemcpyAsync(dlg, dlogits, nlg * 4, hipMemcpyDeviceToDevice, st));
    if (net == 0)
      if (int rc = paig_relu_mask(logits, dlg, nlg, stream)) return rc;
    written[p.LG].push_back({0, K});
    first = no - 1;
  }
  auto state = [&](const Reg& r) {
    int cov = 0;
    for (auto& s : written[r.buf]) {
      const int lo = r.off > s.first ? r.off : s.first, hi = r.off + r.n < s.first + s.second ? r.off + r.n
                                                                                           : s.first + s.second;
      if (hi > lo) cov += hi - lo;
    }
    return cov == 0 ? 0 : (cov == r.n ? 1 : -1);   // 0 write, 1 accumulate, -1 partial (plan error)
  };
  auto mark = [&](const Reg& r) { written[r.buf].push_back({r.off, r.n}); };
  std::vector<const float*> s_src;
  std::vector<int> s_nb, s_len;
  std::vector<float*> s_dst;
  std::vector<bool> folded_up(no, false);
  for (int i = first; i >= 0; --i) {
    if (folded_up[i]) continue;
    const UOp& op = p.ops[i];
    if (op.kind == U_POOL && L.pcode[i] != (size_t)-1) continue;   // folded into the pooled conv's backward
    bool relu_fin = false;
    for (auto& f : p.fin[i]) relu_fin = relu_fin || f.second;
    const View dyv = dview(op.dst);
    int rc = 0;
    if (op.kind == U_CONV) {
      int slvl, xfl = 0;
      View sv;
      if (p.fused_up[i] >= 0) {
        sv = view(p.ops[p.fused_up[i]].src, slvl);
        slvl /= 2;
        xfl = 32;
      } else {
        sv = view(op.src, slvl);
      }
      const int Hl = H / slvl, cin = op.src.n, cout = op.dst.n, ks = op.ks;
      float* slab = reinterpret_cast<float*>(base + L.slab[i]);
      const int n_w = cout * cin * ks * ks;
      int nb = 0;
      const float* xm = xmax + (size_t)i * PAIG_XMAX_SLOTS;
      const void* wp1 = cm != 128 || op.src.buf == p.X0 ? nullptr : (ext ? wpd[op.conv] : base + L.wprep1[i]);
      if (xfl && cm && !sep && paig_conv2d_bwd_supported(cin, cout, Hl, Hl, ks, cm | 32)) {
        // fused-upsample input: the layer backward and the upsample's backward in one launch
        const int ui = p.fused_up[i];
        const Reg usrc = p.ops[ui].src;
        const View dxv = dview(usrc);
        PAIG_REQUIRE(state(usrc) == 0, "paig_unet_bwd: upsample source gradient already written (op %d)", i);
        int flags2 = cm | 32, alvl;
        const float* aux = nullptr;
        long long aux_fs = 0;
        for (auto& f : p.fin[ui])
          if (f.first == usrc && f.second) {
            const View a = view(usrc, alvl);
            aux = a.p;
            aux_fs = a.fs;
            flags2 |= 2;
          }
        pr(0, i, op.conv, PAIG_PROBE_CONV_BWD, cin, cout, Hl, flags2);
        rc = paig_conv2d_bwd(sv.p, sv.fs, sv.grp, sv.gs, dyv.p, dyv.fs, const_cast<float*>(dxv.p), dxv.fs, aux, aux_fs,
                             w[op.conv], slab, NBLK_MAX, &nb, F, cin, cout, Hl, Hl, ks, flags2, xm, PAIG_XMAX_SLOTS,
                             nullptr, 0, nullptr, 0, wp1, stream);
        pr(1, i, op.conv, PAIG_PROBE_CONV_BWD, cin, cout, Hl, flags2);
        if (rc) return rc;
        s_src.push_back(slab), s_nb.push_back(nb), s_len.push_back(n_w + cout), s_dst.push_back(dwb[op.conv]);
        mark(usrc);
        folded_up[ui] = true;
        continue;
      }
      if (op.src.buf != p.X0 && !xfl && cm && !sep && paig_conv2d_bwd_supported(cin, cout, Hl, Hl, ks, cm)) {
        // data and weight gradients in one launch
        const View dxv = dview(op.src);
        const int mode = state(op.src);
        PAIG_REQUIRE(mode >= 0, "paig_unet_bwd: partially written gradient region (op %d)", i);
        int flags2 = cm | (mode == 1 ? 4 : 0), alvl;
        const float* aux = nullptr;
        long long aux_fs = 0;
        if (relu_fin) {
          PAIG_REQUIRE(p.fin[i].size() == 1 && p.fin[i][0].first == op.src, "paig_unet_bwd: mixed ReLU (op %d)", i);
          const View a = view(op.src, alvl);
          aux = a.p;
          aux_fs = a.fs;
          flags2 |= 2;
        }
        const float* dpool = nullptr;
        long long dpool_fs = 0;
        const unsigned char* pcode = nullptr;
        long long pcode_fs = 0;
        if (i + 1 < no && L.pcode[i + 1] != (size_t)-1) {   // the max pool of this output, folded
          // the kernel reads this output's skip-path gradient (dY): the
          // concat partner must have written it
          PAIG_REQUIRE(state(op.dst) == 1, "paig_unet_bwd: pool fold before the skip gradient (op %d)", i);
          const View pdv = dview(p.ops[i + 1].dst);
          dpool = pdv.p;
          dpool_fs = pdv.fs;
          pcode = reinterpret_cast<const unsigned char*>(base + L.pcode[i + 1]);
          pcode_fs = L.pcode_fs[i + 1];
          flags2 |= 64;
        }
        pr(0, i, op.conv, PAIG_PROBE_CONV_BWD, cin, cout, Hl, flags2);
        rc = paig_conv2d_bwd(sv.p, sv.fs, sv.grp, sv.gs, dyv.p, dyv.fs, const_cast<float*>(dxv.p), dxv.fs, aux, aux_fs,
                             w[op.conv], slab, NBLK_MAX, &nb, F, cin, cout, Hl, Hl, ks, cm | (flags2 & 70), xm,
                             PAIG_XMAX_SLOTS, dpool, dpool_fs, pcode, pcode_fs, wp1, stream);
        pr(1, i, op.conv, PAIG_PROBE_CONV_BWD, cin, cout, Hl, flags2);
        if (rc) return rc;
        s_src.push_back(slab), s_nb.push_back(nb), s_len.push_back(n_w + cout), s_dst.push_back(dwb[op.conv]);
        mark(op.src);
        continue;
      }
      // the max pool of this output folded into both launches' dY staging
      // (pool_fold_split): the pooled gradient and the forward's codes
      const bool pf = !xfl && i + 1 < no && L.pcode[i + 1] != (size_t)-1;
      const float* dpool = nullptr;
      long long dpool_fs = 0;
      const unsigned char* pcode = nullptr;
      long long pcode_fs = 0;
      if (pf) {
        PAIG_REQUIRE(state(op.dst) == 1, "paig_unet_bwd: pool fold before the skip gradient (op %d)", i);
        const View pdv = dview(p.ops[i + 1].dst);
        dpool = pdv.p;
        dpool_fs = pdv.fs;
        pcode = reinterpret_cast<const unsigned char*>(base + L.pcode[i + 1]);
        pcode_fs = L.pcode_fs[i + 1];
      }
      pr(0, i, op.conv, PAIG_PROBE_CONV_WGRAD, cin, cout, Hl, xfl | cm | (pf ? 64 : 0));
      rc = pf ? paig_conv2d_wgrad_pf(sv.p, sv.fs, sv.grp, sv.gs, dyv.p, dyv.fs, dpool, dpool_fs, pcode, pcode_fs, slab,
                                     NBLK_MAX, &nb, F, cin, cout, Hl, Hl, ks, cm | 64, xm, PAIG_XMAX_SLOTS, stream)
              : paig_conv2d_wgrad_ex(sv.p, sv.fs, sv.grp, sv.gs, dyv.p, dyv.fs, slab, NBLK_MAX, &nb, F, cin, cout, Hl, Hl,
                                     ks, xfl | cm, xm, PAIG_XMAX_SLOTS, stream);
      pr(1, i, op.conv, PAIG_PROBE_CONV_WGRAD, cin, cout, Hl, xfl | cm | (pf ? 64 : 0));
      if (rc) return rc;
      s_src.push_back(slab), s_nb.push_back(nb), s_len.push_back(n_w + cout), s_dst.push_back(dwb[op.conv]);
      PAIG_REQUIRE(!pf || op.src.buf != p.X0, "paig_unet_bwd: pool fold on the input layer (op %d)", i);
      if (op.src.buf == p.X0) continue;   // no input gradient (Q10)
      const int ui = p.fused_up[i];
      if (ui >= 0 && cm == 128 && !(flags & PAIG_UNET_STANDALONE_UP) &&
          paig_conv2d_mfma_supported(0, cout, cin, Hl, Hl, ks, 8 | 128 | 512)) {
        // the dgrad writes the upsample SOURCE's gradient: the upsample's
        // backward in its epilogue (one launch, no full-resolution gradient)
        const Reg usrc = p.ops[ui].src;
        const View dxv = dview(usrc);
        PAIG_REQUIRE(state(usrc) == 0, "paig_unet_bwd: upsample source gradient already written (op %d)", i);
        int flags2 = 8 | 512, alvl;
        const float* aux = nullptr;
        long long aux_fs = 0;
        for (auto& f : p.fin[ui])
          if (f.first == usrc && f.second) {
            const View a = view(usrc, alvl);
            aux = a.p;
            aux_fs = a.fs;
            flags2 |= 2;
          }
        pr(0, i, op.conv, PAIG_PROBE_CONV_DGRAD, cin, cout, Hl, flags2 | cm);
        rc = paig_conv2d_fwd_pw(dyv.p, dyv.fs, 0, 0, const_cast<float*>(dxv.p), dxv.fs, aux, aux_fs, w[op.conv],
                                nullptr, F, cout, cin, Hl, Hl, ks, flags2 | cm, nullptr, 0, nullptr, 0, wp1, stream);
        pr(1, i, op.conv, PAIG_PROBE_CONV_DGRAD, cin, cout, Hl, flags2 | cm);
        if (rc) return rc;
        mark(usrc);
        folded_up[ui] = true;
        continue;
      }
      const View dxv = dview(op.src);
      const int mode = state(op.src);
      PAIG_REQUIRE(mode >= 0, "paig_unet_bwd: partially written gradient region (op %d)", i);
      int flags2 = 8 | (mode == 1 ? 4 : 0), alvl;
      const float* aux = nullptr;
      long long aux_fs = 0;
      if (relu_fin) {
        PAIG_REQUIRE(p.fin[i].size() == 1 && p.fin[i][0].first == op.src, "paig_unet_bwd: mixed ReLU (op %d)", i);
        const View a = view(op.src, alvl);
        aux = a.p;
        aux_fs = a.fs;
        flags2 |= 2;
      }
      if (pf) flags2 |= 64;
      pr(0, i, op.conv, PAIG_PROBE_CONV_DGRAD, cin, cout, Hl, flags2 | cm);
      rc = paig_conv2d_fwd_pwc(dyv.p, dyv.fs, 0, 0, const_cast<float*>(dxv.p), dxv.fs, aux, aux_fs, w[op.conv], nullptr,
                               F, cout, cin, Hl, Hl, ks, flags2 | cm, nullptr, 0, const_cast<float*>(dpool), dpool_fs,
                               const_cast<unsigned char*>(pcode), pcode_fs, wp1, stream);
      pr(1, i, op.conv, PAIG_PROBE_CONV_DGRAD, cin, cout, Hl, flags2 | cm);
      mark(op.src);
    } else if (op.kind == U_POOL) {
      int slvl;
      const View sv = view(op.src, slvl);
      const int Hl = H / slvl;
      const View dxv = dview(op.src);
      PAIG_REQUIRE(state(op.src) == 1, "paig_unet_bwd: max-pool backward before its concat partner (op %d)", i);
      rc = paig_maxpool2_bwd_relu(sv.p, sv.fs, dyv.p, dyv.fs, const_cast<float*>(dxv.p), dxv.fs, F, op.src.n, Hl, Hl,
                                  stream);
      mark(op.src);
    } else {
      int slvl, dlvl;
      const View sv = view(op.src, slvl);
      (void)view(op.dst, dlvl);
      const int Hs = H / slvl, Ho = H / dlvl;
      const View dxv = dview(op.src);
      PAIG_REQUIRE(state(op.src) == 0, "paig_unet_bwd: upsample source gradient already written (op %d)", i);
      bool relu = false;
      for (auto& f : p.fin[i]) relu = relu || (f.first == op.src && f.second);
      rc = paig_upsample2_bwd(dyv.p, dyv.fs, sv.p, sv.fs, const_cast<float*>(dxv.p), dxv.fs, F, op.src.n, Hs, Hs, Ho,
                              Ho, relu ? 1 : 0, stream);
      mark(op.src);
    }
    if (rc) return rc;
  }
  // every conv's weight + bias gradient and the caller's extra partial-
  // gradient slabs: one batched deterministic reduction
  for (int e = 0; e < n_extra; ++e)
    s_src.push_back(e_src[e]), s_nb.push_back(e_nb[e]), s_len.push_back(e_len[e]), s_dst.push_back(e_dst[e]);
  return paig_slab_reduce_multi((int)s_src.size(), s_src.data(), s_nb.data(), s_len.data(), s_dst.data(), 0, stream);
}

}  // namespace

extern "C" {

size_t paig_unet_workspace_ex(int net, int F, int H, int K, int math, int flags) {
  if (check_args(net, F, H, K, math)) return 0;
  UPlan p;
  build_plan(p, net, K);
  derive(p, H, math);
  ULayout L;
  layout(p, L, F, H, math, flags);
  return L.total;
}

size_t paig_unet_workspace(int net, int F, int H, int K, int math) {
  return paig_unet_workspace_ex(net, F, H, K, math, 0);
}

long long paig_unet_buffer(int net, int F, int H, int K, int math, int flags, int which, int buf) {
  if (check_args(net, F, H, K, math)) return -1;
  UPlan p;
  build_plan(p, net, K);
  derive(p, H, math);
  if (buf < 0 || buf >= (int)p.bufs.size() || (which != 0 && which != 1)) return -1;
  ULayout L;
  layout(p, L, F, H, math, flags);
  const size_t o = which == 0 ? L.act[buf] : L.grad[buf];
  return o == (size_t)-1 ? -1 : (long long)o;
}

int paig_unet_query(int net, int K, int what) {
  if (net != 0 && net != 1) return -1;
  UPlan p;
  build_plan(p, net, K);
  switch (what) {
    case 0: return p.nconv;
    case 1: return (int)p.bufs.size();
    case 2: return p.ops.back().src.buf;   // the 1x1 head's input buffer
    case 3: return p.ops.back().src.n;     // ... and its channels
    case 4: return p.LG;
    case 5: return p.ops.back().src.off;                 // the head input's channel offset in its buffer
    case 6: return p.bufs[p.ops.back().src.buf].C;       // ... and that buffer's channels
    default: return -1;
  }
}

int paig_unet_fwd_ex(int net, int F, int H, int K, int math, int flags, const float* x, long long x_fs, int x_grp,
                     long long x_gs, const float* const* w, const float* const* b, float* logits,
                     const void* const* wprep_fwd, const void* const* wprep_dg, void* ws, size_t ws_bytes,
                     paig_unet_probe_fn probe, void* probe_ctx, void* stream) {
  return fwd_impl(net, F, H, K, math, flags, x, x_fs, x_grp, x_gs, w, b, logits, wprep_fwd, wprep_dg, ws, ws_bytes,
                  UProbe{probe, probe_ctx}, stream);
}

int paig_unet_bwd_ex(int net, int F, int H, int K, int math, int flags, const float* x, long long x_fs, int x_grp,
                     long long x_gs, const float* const* w, const float* logits, const float* dlogits,
                     float* const* dwb, int n_extra, const float* const* extra_src, const int* extra_nblk,
                     const int* extra_len, float* const* extra_dst, const void* const* wprep_dg, void* ws,
                     size_t ws_bytes, paig_unet_probe_fn probe, void* probe_ctx, void* stream) {
  return bwd_impl(net, F, H, K, math, flags, x, x_fs, x_grp, x_gs, w, logits, dlogits, dwb, n_extra, extra_src,
                  extra_nblk, extra_len, extra_dst, wprep_dg, ws, ws_bytes, UProbe{probe, probe_ctx}, stream);
}

int paig_unet_fwd(int net, int F, int H, int K, int math, const float* x, long long x_fs, int x_grp, long long x_gs,
                  const float* const* w, const float* const* b, float* logits, void* ws, size_t ws_bytes,
                  void* stream) {
  return fwd_impl(net, F, H, K, math, 0, x, x_fs, x_grp, x_gs, w, b, logits, nullptr, nullptr, ws, ws_bytes,
                  UProbe{nullptr, nullptr}, stream);
}

int paig_unet_bwd(int net, int F, int H, int K, int math, const float* x, long long x_fs, int x_grp, long long x_gs,
                  const float* const* w, const float* logits, const float* dlogits, float* const* dwb, void* ws,
                  size_t ws_bytes, void* stream) {
  return bwd_impl(net, F, H, K, math, 0, x, x_fs, x_grp, x_gs, w, logits, dlogits, dwb, 0, nullptr, nullptr, nullptr,
                  nullptr, nullptr, ws, ws_bytes, UProbe{nullptr, nullptr}, stream);
}

}  // extern "C"
