"""GPU: the shortened correctly-rounded sequences the kernels use (libm_ref.hpp rcp_rn_normal, div_softsign;
x2_device.hpp rcp2) equal the IEEE results on EVERY float of their domains, checked on the device itself
(v_rcp_f32 is a hardware approximation no host can emulate bit for bit): tools/exhaustive_ops.hip, built by
__graft_entry__.build().  The reference column (the compiler's IEEE sequence) is cross-checked against a
double-precision evaluation rounded once."""
import os
import re
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tools", "exhaustive_ops")


def test_shortened_division_sequences_are_exact_on_their_domains():
    if not os.path.exists(EXE):
        pytest.skip("tools/exhaustive_ops not built (__graft_entry__.build())")
    r = subprocess.run(["timeout", "-k", "10", "120", EXE], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    res = {}
    for line in r.stdout.splitlines():
        m = re.match(r"(\S+)\s+(\S+)\s+inputs (\d+) mismatches (\d+)", line)
        if m:
            res[(m.group(1), m.group(2))] = (int(m.group(3)), int(m.group(4)))
    shipped = [("rcp", "newton+1corr"), ("sqrt", "current"), ("soft+<", "2corr-negres"), ("soft-<", "2corr-negres")]
    for key in shipped + [k for k in res if k[1] == "ref-vs-double"]:
        n, bad = res[key]
        assert n > 100_000_000 and bad == 0, (key, n, bad)
