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


def apply(csrc, name):
    for fname, anchor, text, where in ABLATIONS[name]:
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
    if len(sys.argv) < 3 or any(n not in ABLATIONS for n in sys.argv[2:]):
        raise SystemExit("usage: ablations.py <csrc_dir> <name>...; names: %s" % ", ".join(sorted(ABLATIONS)))
    for n in sys.argv[2:]:
        apply(sys.argv[1], n)
