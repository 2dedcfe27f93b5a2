#!/usr/bin/env python3
"""Ablation builds: parity-breaking source edits applied to a COPY of the library's sources, for attributing kernel
time (never part of the shipped library; tools/build_variant.sh applies them).

    python tools/ablations.py <csrc_dir> <name> [<name> ...]

Each ablation is a list of (file, anchor, text, where): `text` is inserted before or after the unique `anchor`, or
replaces it; a
missing or repeated anchor fails loudly (the sources moved on and the ablation needs updating).
"""
import os
import sys

ABLATIONS = {
    # SW checkpointed solver: stop after pass 1, or after pass 2 (pass times by difference)
    "swck_pass1": [("kernels_sw_ck.hip", "  // ---- pass 2: bottom -> top adding; albedo / source checkpoint",
                    "  return;  // ablation swck_pass1\n", "before")],
    "swck_pass12": [("kernels_sw_ck.hip", "  // ---- pass 3: top -> bottom fluxes + ordered broadband sums ----",
                     "  return;  // ablation swck_pass12\n", "before")],
    # SW checkpointed solver: no ordered broadband flush (ring written, never summed)
    "swck_noflush": [("kernels_sw_ck.hip", "  auto flush = [&](int n, int lev0, int dl, int slot0 = 0) {\n",
                      "    return;  // ablation swck_noflush\n", "after")],
    # MLP (16x16x4 kernel): hidden activations x/2 instead of softsign
    "mlp_cheap_act": [("kernels_nn.hip", "  if constexpr (ACTS == 1) return softsign(x);",
                       "  if constexpr (ACTS == 1) return x * 0.5f;  // ablation mlp_cheap_act\n", "before")],
    # MLP on 32x32x2 tiles: LW pair stores dropped unless a value is a nan
    "mlp32_nostore": [("kernels_nn32.hip", "const float tau = pow8(t) * cdr[r], pf = p * p;\n          const uint32_t off = vo[r] + 128u * go;\n",
                       "const float tau = pow8(t) * cdr[r], pf = p * p;\n"
                       "          const uint32_t off = (tau != tau || pf != pf) ? vo[r] + 128u * go : kOOB;"
                       "  // ablation mlp32_nostore\n", "replace")],
}

ABLATIONS.update({
    # SW pair (32x32x2 kernel): stores dropped unless a value is a nan (the write path's share of the kernel)
    "mlp32_sw_nostore": [("kernels_nn32.hip", """          const uint32_t off = vo[r] + 128u * go;
          o0.st(tot, off);
          o1.st(ssa, off);""", """          const uint32_t off = (tot != tot || ssa != ssa) ? vo[r] + 128u * go : kOOB;  // ablation mlp32_sw_nostore
          o0.st(tot, off);
          o1.st(ssa, off);""", "replace")],
    # SW pair: the same bytes as 16-byte stores (lane (c, h) writes 16 bytes of row 8b + 4h + (c >> 3) at g-point
    # 32go + 4(c & 7): 4 dwordx4 per array and g-tile instead of 16 dwords) -- values scrambled, addresses and widths
    # those of a transposed epilogue (the store width's share of the kernel)
    "mlp32_sw_st4": [("kernels_nn32.hip", """          const uint32_t off = vo[r] + 128u * go;
          o0.st(tot, off);
          o1.st(ssa, off);
        }""", """          tots[r] = tot;
          ssas[r] = ssa;
        }
#pragma unroll
        for (int b = 0; b < 4; b++) {  // ablation mlp32_sw_st4
          const uint32_t R = 8u * b + 4u * h + ((uint32_t)j >> 3);
          const uint32_t off = R < nvalid ? 4u * (R * (uint32_t)ngpt) + 128u * go + 16u * ((uint32_t)j & 7u) : kOOB;
          o0.st4((floatx4){tots[4 * b], tots[4 * b + 1], tots[4 * b + 2], tots[4 * b + 3]}, off);
          o1.st4((floatx4){ssas[4 * b], ssas[4 * b + 1], ssas[4 * b + 2], ssas[4 * b + 3]}, off);
        }""", "replace"),
                     ("kernels_nn32.hip", """        const float bB = iB[LB.b3 + g], sdB = iB[LB.sd + g], mnB = iB[LB.mn + g];
#pragma unroll
        for (int r = 0; r < 16; r++) {
          float ta""", """        const float bB = iB[LB.b3 + g], sdB = iB[LB.sd + g], mnB = iB[LB.mn + g];
        float tots[16], ssas[16];
#pragma unroll
        for (int r = 0; r < 16; r++) {
          float ta""", "replace")],
})

ABLATIONS.update({
    # SW pair: the epilogue's arithmetic replaced by the raw network outputs (stores kept): its VALU share
    "mlp32_sw_noepi": [("kernels_nn32.hip", """          float ta = sdA * (yA[r] + bA);
          ta = ta + mnA;
          const float vabs = pow8(ta) * cdr[r];
          float tr = sdB * (yB[r] + bB);
          tr = tr + mnB;
          const float vray = pow8(tr) * cdr[r];
          const float tot = vabs + vray, ssa = vray / tot;""", """          const float tot = yA[r], ssa = yB[r];  // ablation mlp32_sw_noepi""", "replace")],
    # every network's output-layer MFMA chains skipped (zero accumulators): their share
    "mlp32_noout": [("kernels_nn32.hip", """      const floatx16 yA = mfma_chain_t<AN3>(iA + LA.l3, go, hA, lane);
      floatx16 yB = {};
      if constexpr (kPair) yB = mfma_chain_t<BN3>(iB + LB.l3, go, hB, lane);""", """      floatx16 yA = {}, yB = {};  // ablation mlp32_noout
      yA[0] = hA[0];
      if constexpr (kPair) yB[0] = hB[0];""", "replace")],
})

_LW_UP = """          const float T = solver_exp_neg(-t, etab);
          const float fact = (t > tau_thresh) ? solver_div(1.0f - T, t) - T : t * (0.5f - 1.0f / 3.0f * t);
          const float S = (1.0f - T) * lvup"""
ABLATIONS.update({
    # LW no-scattering solver: the up pass without its exp (T from a cheap stand-in), or without exp and division --
    # the share a down-pass cache of the transmittance (and of fact) could save
    "lw_up_noexp": [("kernels_rte.hip", _LW_UP, _LW_UP.replace("solver_exp_neg(-t, etab)", "1.0f - 0.5f * t")
                     + "  /* ablation lw_up_noexp */", "replace")],
    "lw_up_noexpdiv": [("kernels_rte.hip", _LW_UP, _LW_UP.replace("solver_exp_neg(-t, etab)", "1.0f - 0.5f * t")
                        .replace("solver_div(1.0f - T, t)", "(1.0f - T) * t") + "  /* ablation lw_up_noexpdiv */",
                        "replace")],
})

# Variants that keep the bits (tools/kernel_ab.py checks them bitwise against the default library): A/B candidates
ABLATIONS.update({
    # SW checkpointed solver: scheduling fences between a pass's chunk bodies and their prefetches (rounds 2-3)
    "swck_fence": [("kernels_sw_ck.hip", """      load(B, idx(min(i + 1, count - 1)));
      body(A, idx(i), true);
      load(A, idx(min(i + 2, count - 1)));
""", """      load(B, idx(min(i + 1, count - 1)));
      __builtin_amdgcn_sched_barrier(0);
      body(A, idx(i), true);
      load(A, idx(min(i + 2, count - 1)));
      __builtin_amdgcn_sched_barrier(0);
""", "replace")],
})


ABLATIONS.update({
    # VALU attribution (round 6, C5): every solver exp on the hardware exponential -- the direct-beam transmittance too
    # (build with -DRRTMGPNN_FAST_LIBM=1, which already does the rest); the exps' share of SQ_INSTS_VALU by difference
    "exp_hw_all": [("rte_device.hpp",
                    "__device__ __forceinline__ float solver_exp_beam(float x, const uint64_t *tab) { return ref_expf_neg(x, tab); }",
                    "__device__ __forceinline__ float solver_exp_neg(float x, const uint64_t *tab);\n"
                    "__device__ __forceinline__ float solver_exp_beam(float x, const uint64_t *tab) { return solver_exp_neg(x, tab); }"
                    "  // ablation exp_hw_all", "replace"),
                   ("x2_device.hpp", """  constexpr int L = sizeof(V) / sizeof(float);
  float xs[N * L], ys[N * L];
#pragma unroll
  for (int i = 0; i < N; i++) __builtin_memcpy(&xs[i * L], &x[i], sizeof(V));
  ref_expf_neg_batch<N * L>(xs, ys, etab);
#pragma unroll
  for (int i = 0; i < N; i++) __builtin_memcpy(&y[i], &ys[i * L], sizeof(V));
}

// 8-byte""", """#pragma unroll
  for (int i = 0; i < N; i++) y[i] = exp2v_beam(x[i], etab);  // ablation exp_hw_all
}

// 8-byte""", "replace")],
    # VALU attribution: the solvers' correctly rounded divisions, reciprocals and square roots as the bare hardware
    # estimates (v_rcp_f32, v_sqrt_f32): their share of SQ_INSTS_VALU by difference
    "div_hw": [("libm_ref.hpp", """  float r = __builtin_amdgcn_rcpf(b);
  r = fmaf(fmaf(-b, r, 1.0f), r, r);
  return fmaf(fmaf(-b, r, 1.0f), r, r);
}""", """  return __builtin_amdgcn_rcpf(b);  // ablation div_hw
}""", "replace"),
               ("libm_ref.hpp", """  float r = __builtin_amdgcn_rcpf(b);
  r = fmaf(fmaf(-b, r, 1.0f), r, r);
  float q = a * r;
  q = fmaf(fmaf(-b, q, a), r, q);
  return fmaf(fmaf(-b, q, a), r, q);
}""", """  return a * __builtin_amdgcn_rcpf(b);  // ablation div_hw
}""", "replace"),
               ("libm_ref.hpp", """  const float s = __builtin_amdgcn_sqrtf(x);
  const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
  const float em = fmaf(-sm, s, x), ep = fmaf(-sp, s, x);
  float r = (em <= 0.0f) ? sm : s;
  return (ep > 0.0f) ? sp : r;
}""", """  return __builtin_amdgcn_sqrtf(x);  // ablation div_hw
}""", "replace"),
               ("x2_device.hpp", """  const f2 s = (f2){__builtin_amdgcn_sqrtf(x.x), __builtin_amdgcn_sqrtf(x.y)};
  const f2 sm""", """  return (f2){__builtin_amdgcn_sqrtf(x.x), __builtin_amdgcn_sqrtf(x.y)};  // ablation div_hw
  const f2 s = (f2){__builtin_amdgcn_sqrtf(x.x), __builtin_amdgcn_sqrtf(x.y)};
  const f2 sm""", "replace"),
               ("x2_device.hpp", """  f2 r = (f2){__builtin_amdgcn_rcpf(b.x), __builtin_amdgcn_rcpf(b.y)};
  const f2 one = splat(1.0f);""", """  f2 r = (f2){__builtin_amdgcn_rcpf(b.x), __builtin_amdgcn_rcpf(b.y)};
  return r;  // ablation div_hw
  const f2 one = splat(1.0f);""", "replace"),
               ("x2_device.hpp", """  f2 r = (f2){__builtin_amdgcn_rcpf(b.x), __builtin_amdgcn_rcpf(b.y)};
  r = vfma(vfma(-b, r, splat(1.0f)), r, r);
  f2 q = a * r;""", """  f2 r = (f2){__builtin_amdgcn_rcpf(b.x), __builtin_amdgcn_rcpf(b.y)};
  return a * r;  // ablation div_hw
  f2 q = a * r;""", "replace")],
})


def parametric(name):
    """swck_small:K:R:W -- the small-grid SW instance's chunk length, ring levels and wave floor;
    swck_planes:T:E -- its beam-transmittance (T) and exp(-k tau) (E) workspace planes on (1) or off (0);
    swck_big:K:R:W -- the large-grid instances' chunk length, ring levels and wave floor (the all-sky ones; C4);
    swck_nnw:W -- the large-grid clear-sky (NN) instance's wave floor (C5);
    swck_nnplanes:T:E / swck_incplanes:T:E -- the same planes in the large-grid clear-sky (C5) / all-sky (C4)
    instances;
    mlp_sw:NT:W -- the SW network's threads per block and waves-per-SIMD floor (kernels_nn32.hip).
    (The LW network's grid cap is a library call now, rrtmgpnn_context_set_mlp_max_cus / bench.py --lw-net-cus.)"""
    f = name.split(":")
    if f[0] == "swck_small" and len(f) == 4:
        return [("kernels_sw_ck.hip", None, "constexpr int kCkKSmall = %s, kCkRingSmall = %s, kCkWavesSmall = %s;"
                 % tuple(f[1:]), r"constexpr int kCkKSmall = \d+, kCkRingSmall = \d+, kCkWavesSmall = \d+;")]
    if f[0] == "swck_big" and len(f) == 4:
        return [("kernels_sw_ck.hip", None, "constexpr int kCkK = %s, kCkRing = %s, kCkWaves = %s;" % tuple(f[1:]),
                 r"constexpr int kCkK = \d+, kCkRing = \d+, kCkWaves = \d+;")]
    if f[0] == "swck_nnw" and len(f) == 2:
        return [("kernels_sw_ck.hip", None, "constexpr int kCkWavesNN = %s;" % f[1],
                 r"constexpr int kCkWavesNN = \d+;")]
    if f[0] == "mlp_packin" and len(f) == 2:
        return [("kernels_nn32.hip", None, "constexpr bool kMlpPackedIn = %s;" % ("true" if f[1] == "1" else "false"),
                 r"constexpr bool kMlpPackedIn = \w+;")]
    if f[0] == "mlp_stagger" and len(f) == 3:  # waves >= 4 of a block start N x 64 cycles late, at priority P
        code = "  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nwaves = blockDim.x >> 6;\n"
        extra = ""
        if int(f[1]) > 0:
            extra += "  if (wave >= 4) { for (int i_ = 0; i_ < %d; i_++) __builtin_amdgcn_s_sleep(32); }\n" % (int(f[1]) // 32)
        if int(f[2]) > 0:
            extra += "  if (wave >= 4) __builtin_amdgcn_s_setprio(%d);\n" % int(f[2])
        return [("kernels_nn32.hip", code, extra, "after")]
    if f[0] == "lw_ldspad" and len(f) == 2:  # the LW solver's blocks hold KB more LDS each (fewer blocks per CU)
        return [("kernels_rte.hip", "  extern __shared__ __attribute__((aligned(16))) float smem[];\n  const int icol = blockIdx.x, g = threadIdx.x;\n",
                 "  __shared__ float pad_[%d * 256];\n  if (ngpt == -12345) { pad_[threadIdx.x] = 1.0f; flux_up[0] = pad_[threadIdx.x ^ 1]; }\n"
                 % int(f[1]), "after")]
    if f[0] == "mlp_lw" and len(f) == 3:  # the fused LW pair's threads per block and waves-per-SIMD floor
        return [("kernels_nn32.hip", "return launch32<9, 2, 29, 2, 29, 1, 8, 1, 8, 8, MLP_LW_PAIR, true>(ctx, a);",
                 "return launch32<9, 2, 29, 2, 29, 1, 8, 1, 8, 8, MLP_LW_PAIR, true, %s, %s>(ctx, a);" % tuple(f[1:]),
                 "replace")]
    if f[0] == "mlp_unroll" and len(f) == 2:  # output g-tiles per unrolled step (both pairs)
        return [("kernels_nn32.hip", "#pragma unroll 1\n    for (int go = 0; go < NGT; go++) out_tile(go);",
                 "#pragma unroll %s\n    for (int go = 0; go < NGT; go++) out_tile(go);" % f[1], "replace")]
    if f[0] == "flush_unroll" and len(f) == 3:  # the ordered flushes' loads in flight: LW (ring_flush_lanes), SW
        return [("rte_device.hpp", "#pragma unroll 8\n    for (int m = 0; m < n4; m++) sum = sum + r[4 * m];\n    part[",
                 "#pragma unroll %s\n    for (int m = 0; m < n4; m++) sum = sum + r[4 * m];\n    part[" % f[1], "replace"),
                ("rte_device.hpp", """#pragma unroll 8
      for (int m = 0; m < n4; m++) sum = (sum + r[4 * m]) + r2[4 * m];
    } else {
#pragma unroll 8
      for (int m = 0; m < n4; m++) sum = sum + r[4 * m];""", """#pragma unroll %s
      for (int m = 0; m < n4; m++) sum = (sum + r[4 * m]) + r2[4 * m];
    } else {
#pragma unroll %s
      for (int m = 0; m < n4; m++) sum = sum + r[4 * m];""" % (f[2], f[2]), "replace")]
    if f[0] == "swck_ahead" and len(f) == 2:
        return [("kernels_sw_ck.hip", None, "constexpr int kCkAheadSmall = %s;" % f[1], r"constexpr int kCkAheadSmall = \d+;")]
    if f[0] == "swck_p1small" and len(f) == 2:
        return [("kernels_sw_ck.hip", None, "constexpr int kCkP1Small = %s;" % f[1], r"constexpr int kCkP1Small = \d+;")]
    if f[0] == "swck_vsmall" and len(f) == 2:
        return [("kernels_sw_ck.hip", None, "using VSmall = %s;" % f[1], r"using VSmall = \w+;")]
    if f[0] in ("swck_nnplanes", "swck_incplanes") and len(f) == 3:
        t, e = ("true" if v == "1" else "false" for v in f[1:])
        suf = "NN" if f[0] == "swck_nnplanes" else "Inc"
        return [("kernels_sw_ck.hip", None, "constexpr bool kCkTn%s = %s, kCkEmk%s = %s;" % (suf, t, suf, e),
                 r"constexpr bool kCkTn%s = \w+, kCkEmk%s = \w+;" % (suf, suf))]
    if f[0] == "mlp_sw" and len(f) == 3:
        return [("kernels_nn32.hip", None, "constexpr int kMlp32Threads = 512, kSwNT = %s, kSwWPE = %s;" % tuple(f[1:]),
                 r"constexpr int kMlp32Threads = 512, kSwNT = \d+, kSwWPE = \d+;")]
    if f[0] == "swck_planes" and len(f) == 3:
        t, e = ("true" if v == "1" else "false" for v in f[1:])
        return [("kernels_sw_ck.hip", None, "constexpr bool kCkTnSmall = %s, kCkEmkSmall = %s;" % (t, e),
                 r"constexpr bool kCkTnSmall = \w+, kCkEmkSmall = \w+;")]
    return None


def apply(csrc, name):
    edits = ABLATIONS.get(name) or parametric(name)
    for fname, anchor, text, where in edits:
        if anchor is None:  # parametric: `where` is a regex matching exactly one line
            import re
            path = os.path.join(csrc, fname)
            with open(path) as f:
                src = f.read()
            new, n = re.subn(where, text, src)
            if n != 1:
                raise SystemExit("ablation %s: pattern matched %d times in %s" % (name, n, fname))
            with open(path, "w") as f:
                f.write(new)
            continue
        path = os.path.join(csrc, fname)
        with open(path) as f:
            src = f.read()
        n = src.count(anchor)
        if n != 1:
            raise SystemExit("ablation %s: anchor found %d times in %s: %r" % (name, n, fname, anchor[:60]))
        src = src.replace(anchor, {"before": text + anchor, "after": anchor + text, "replace": text}[where])
        with open(path, "w") as f:
            f.write(src)


if __name__ == "__main__":
    if len(sys.argv) < 3 or any(n not in ABLATIONS and parametric(n) is None for n in sys.argv[2:]):
        raise SystemExit("usage: ablations.py <csrc_dir> <name>...; names: %s" % ", ".join(sorted(ABLATIONS)))
    for n in sys.argv[2:]:
        apply(sys.argv[1], n)
