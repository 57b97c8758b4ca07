"""Inputs of the golden fixture sets (tests/golden/manifest.json) and the
canonical record-stream digest used by the full-size digests
(tests/golden/full_digests.json).  Generator sets are regenerated from their
seeds; "builder" sets are hand-built batches (tests/batches.py).  Both are
pinned by the sha256 of the packed input bytes."""
from __future__ import annotations

import hashlib

import numpy as np

import libreactorng_amd as rhp
from batches import BUILDERS, pack


def inputs(spec):
    if "builder" in spec:
        buf, off = pack(BUILDERS[spec["builder"]](), align_shift=spec.get("align_shift", 0))
    else:
        buf, off = rhp.generate(spec["config"], spec["n"], spec["seed"], lo=spec.get("lo", 0))
    assert hashlib.sha256(buf.tobytes()).hexdigest() == spec["input_sha256"], "input drifted"
    return buf, off


def record_digest(reqs, hdrs, http=None) -> str:
    """sha256 of a canonical record stream: reqs, then hdrs, then http (rhp.h
    layouts); rhp.record_digest, the one bench.py's parity check uses too."""
    return rhp.record_digest(reqs, hdrs, http)
