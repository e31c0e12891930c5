"""The device graph sampler's stream is pinned to snapshot.SAMPLER_RULE.

A resumed ensemble campaign (snapshot.restore) assumes its remaining trials draw their graphs
from the stream its first part drew from; the snapshot records SAMPLER_RULE for that.  The
device == oracle parity tests cannot notice a stream change that device and oracle make
together, so this test pins digests of the oracle's restatement (one-level and sequential-draw
regimes) together with the rule string: a stream change fails here until SAMPLER_RULE is bumped
and tests/golden/make_sampler_stream.py is re-run."""
import json
import os

import pytest

from iib_project_ldpc_codes_amd import snapshot
from tests.golden.make_sampler_stream import digest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sampler_stream.json")


def _golden():
    with open(GOLDEN) as f:
        return json.load(f)


def test_sampler_rule_matches_pinned_stream():
    assert _golden()["sampler_rule"] == snapshot.SAMPLER_RULE, \
        "SAMPLER_RULE changed: regenerate tests/golden/sampler_stream.json (make_sampler_stream.py)"


@pytest.mark.parametrize("case", _golden()["cases"], ids=lambda c: f"n{c['n']}-s{c['seed']}-g{c['graph']}")
def test_sampler_stream_digest(case):
    got = digest(case["n"], case["seed"], case["graph"])
    assert got == case["sha256"], (
        f"the sampler stream changed for {case} under SAMPLER_RULE {snapshot.SAMPLER_RULE!r}: bump "
        "snapshot.SAMPLER_RULE (resumed campaigns must not mix streams) and re-run tests/golden/make_sampler_stream.py")
