"""Regenerate tests/golden/sampler_stream.json: digests of the oracle's restatement of the device
graph sampler (the stream that decides which graph ensemble trial t decodes), keyed to
snapshot.SAMPLER_RULE.  Run after an intended stream change, together with a SAMPLER_RULE
bump (tests/test_sampler_stream.py fails until both agree):
    python tests/golden/make_sampler_stream.py"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from iib_project_ldpc_codes_amd import snapshot  # noqa: E402
from oracle import oracle  # noqa: E402

# (n, seed, graph): n = 1,000 (E = 3,000) is the one-level Rao-Sandelius regime, n = 10,000 and
# 64,800 (E = 30,000 / 194,400) the sequential-draw regime
CASES = [(1000, 3, 0), (1000, 3, 7), (10000, 5, 0), (64800, 12, 0), (64800, 12, 9), (64800, 41, 3)]


def digest(n, seed, g):
    chk, var, att = oracle.sample_regular(n, 3, 6, seed, g)
    h = hashlib.sha256()
    h.update(chk.tobytes())
    h.update(var.tobytes())
    h.update(int(att).to_bytes(8, "little", signed=True))
    return h.hexdigest()


if __name__ == "__main__":
    out = {"sampler_rule": snapshot.SAMPLER_RULE,
           "cases": [{"n": n, "dv": 3, "dc": 6, "seed": s, "graph": g, "sha256": digest(n, s, g)} for n, s, g in CASES]}
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "sampler_stream.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))
