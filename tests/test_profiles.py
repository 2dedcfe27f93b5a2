"""profiles/ provenance: the counter files bench.py reads by default (profiles/pmc_traffic.json, pmc_sq.json) hold,
for every config, exactly the per-round file their "_source" names (written together by tools/publish_profiles.py),
so every traffic / valu_busy figure a bench line or DESIGN.md quotes reproduces from one committed file."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench_defaults():
    import argparse
    import sys
    sys.path.insert(0, ROOT)
    import bench
    saved = sys.argv
    sys.argv = ["bench.py"]
    try:
        return bench.parse()
    finally:
        sys.argv = saved


@pytest.mark.parametrize("kind,arg", [("pmc_traffic", "traffic_json"), ("pmc_sq", "sq_json")])
def test_bench_counter_files_equal_their_round_files(kind, arg):
    args = _bench_defaults()
    path = getattr(args, arg)
    assert os.path.abspath(path) == os.path.join(ROOT, "profiles", kind + ".json")
    with open(path) as f:
        top = json.load(f)
    cfgs = [k for k in top if not k.startswith("_")]
    assert {"c3", "c4", "c5"} <= set(cfgs)
    src = top.get("_source", {})
    for cfg in cfgs:
        assert cfg in src, "%s: %s has no _source file" % (kind, cfg)
        rel = src[cfg]
        assert rel.startswith("profiles/r") and os.path.exists(os.path.join(ROOT, rel)), rel
        with open(os.path.join(ROOT, rel)) as f:
            assert json.load(f) == top[cfg], "%s[%s] differs from %s" % (kind, cfg, rel)
    # the round these files come from is the newest round directory that holds counter files
    rounds = sorted(d for d in os.listdir(os.path.join(ROOT, "profiles")) if d.startswith("r") and d[1:].isdigit()
                    and any(n.startswith(kind + "_") for n in os.listdir(os.path.join(ROOT, "profiles", d))))
    assert all(src[c].startswith("profiles/%s/" % rounds[-1]) for c in cfgs), (src, rounds[-1])
