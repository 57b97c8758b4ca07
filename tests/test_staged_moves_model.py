"""A CPU model of rhp_kernel.hip's staged_moves -- the wave's payload moves of
chunked bodies (http.c:134-160, the memmove of each chunk's data down to the
running body end): per body the framed bytes as 16-byte lines into an LDS slot,
then per lane the 16-byte block of the de-framed body: five slot dwords read at
the lane's own byte position for the chunk holding the block's first byte
(funnel-shifted), the bytes from the next chunk's start on taken the same way
from that chunk (and from every later chunk that starts inside the block).  The
same arithmetic, lane by lane, over the chunked workload's bodies that the
kernel stages (<= 8 chunks, lead + framed bytes + 20 <= 2048): the blocks
rebuild exactly the oracle's de-framed bytes, every global load stays inside
the body's framed lines, every slot read inside the slot, and a store leaves
the body only as a whole line inside the request that rewrites the bytes
around the body with their own values.  The GPU tests check the kernel itself (golden sets and the
full-size digest)."""
import numpy as np

import libreactorng_amd as rhp
from oracle_util import run_oracle

K_MOVE_CHUNKS, K_STAGE_BODY = 8, 2048


def chunk_spans(buf, start, end):
    """[(src, n)] data spans (body-relative) and the framed length up to the last data byte,
    as one_chunk_t walks a valid body"""
    at, out, region = start, [], 0
    while True:
        nl = bytes(buf[at:end]).index(b"\n")
        size = int(bytes(buf[at:at + nl + 1]).split(b";")[0].strip(b" \t\r\n"), 16)
        data = at + nl + 1
        if size == 0:
            return out, region
        out.append((data - start, size))
        region = data - start + size
        at = data + size + 2


def staged_body(buf, base, spans, region, size, req_start):
    """one body: returns the (address, byte) stores and checks every access"""
    la = base & ~15
    lead = base - la
    lines = (base + region + 15 - la) >> 4
    assert lines <= 128
    slot = bytearray(K_STAGE_BODY)
    for lane in range(64):
        for h in range(2):
            line = lane + 64 * h
            a = la + (16 * line if line < lines else 0)
            assert la <= a and a + 16 <= la + 16 * max(lines, 1), "a global load outside the body's lines"
            slot[16 * line:16 * line + 16] = bytes(buf[a:a + 16])
    nch = len(spans)
    cd, dl = [0], []
    for cs, n in spans:
        dl.append(cs - cd[-1])
        cd.append(cd[-1] + n)
    L = cd[-1]

    def fetch(P):
        assert 0 <= P and (P & ~3) + 20 <= K_STAGE_BODY, "a slot read outside the slot"
        return slot[P:P + 16]

    stores = []
    for b in range((lead + L + 15) >> 4):
        t0 = 16 * b - lead
        c = max([j for j in range(nch) if j == 0 or cd[j] <= t0])
        out = bytearray(fetch(16 * b + dl[c]))
        for j in range(c + 1, nch):   # every later chunk that starts inside the block, in order
            if cd[j] < t0 + 16:
                out[cd[j] - t0:] = fetch(16 * b + dl[j])[cd[j] - t0:]
        A = la + 16 * b
        kb, ke = max(-t0, 0), min(L - t0, 16)
        if (0 <= t0 and t0 + 16 <= L) or t0 + 16 <= size:
            # a whole line: the bytes outside the body from the slot (the line as it is in memory),
            # all of them inside this request
            for k in range(16):
                v = out[k] if kb <= k < ke else slot[16 * b + k]
                assert req_start <= A + k < base + size, "a whole-line store outside the request"
                if not kb <= k < ke:
                    assert v == buf[A + k], "a byte around the body changed"
                stores.append((A + k, v))
        else:
            for k in range(kb, ke):
                assert base <= A + k < base + L, "a store outside the body"
                stores.append((A + k, out[k]))
    return stores


def test_staged_moves_model_matches_oracle():
    n = 2048
    buf, off = rhp.generate(rhp.GEN_CHUNKED, n, 4242)
    reqs, _, http, want = run_oracle(buf, off, 16, rhp.MODE_HTTP)
    work = buf.copy()
    staged = 0
    for i in range(n):
        if http["result"][i] != 1 or not http["body_kind"][i]:
            continue
        base, end = int(off[i]) + int(reqs["ret"][i]), int(off[i + 1])
        spans, region = chunk_spans(buf, base, end)
        L = sum(x for _, x in spans)
        if len(spans) > K_MOVE_CHUNKS or (base & 15) + region + 20 > K_STAGE_BODY:
            work[base:base + L] = want[base:base + L]   # the kernel's per-thread mover
            continue
        staged += 1
        for a, v in staged_body(buf, base, spans, region, end - base, int(off[i])):   # every load before any store
            work[a] = v
    assert staged > n * 0.8
    assert np.array_equal(work, want), f"{int((work != want).sum())} bytes differ from the oracle's"


K_STAGE_BODIES = 4


def group_schedule(m):
    """rhp_kernel.hip staged_moves' hand-out, step by step: take() fills the
    four slots of a group from the lowest set bits of the mask m (a slot with
    no body left gets have bit 0 and the group's first owner, which is a valid
    lane whenever any slot holds a body; an all-empty group's owners stay
    unset: None here), the loop loads a group only when it holds a body and
    ends at the first empty one.  Returns the groups as (owners, have) in
    processing order, asserting what the kernel relies on."""
    groups = []

    def take(prev_owner0):
        nonlocal m
        owner, have = [None] * K_STAGE_BODIES, 0
        for q in range(K_STAGE_BODIES):
            owner[q] = (m & -m).bit_length() - 1 if m else (owner[0] if q else prev_owner0)
            if m:
                have |= 1 << q
            m &= (m - 1) if m else 0
        return owner, have

    g = take(None)   # the call site runs staged_moves only for m != 0
    assert g[1], "the first group holds a body"
    while g[1]:
        groups.append(g)
        gn = take(None)   # the kernel's Group gn is fresh: an empty group's owner[0] is unset (never read)
        g = gn
    return groups


def test_staged_moves_group_take_model():
    rng = np.random.default_rng(7)
    masks = [1, 1 << 63, (1 << 64) - 1, 0b1011, 0b1111, 0b11111, (1 << 63) | 1, 0x8000_0000_0000_0007]
    masks += [int(rng.integers(1, 1 << 63)) | (int(rng.integers(0, 2)) << 63) for _ in range(2000)]
    masks += [(1 << k) - 1 for k in range(1, 65)] + [((1 << k) - 1) << (64 - k) for k in range(1, 65)]
    for m0 in masks:
        lanes = [j for j in range(64) if m0 >> j & 1]
        groups = group_schedule(m0)
        taken = []
        for owner, have in groups:
            assert have & (have + 1) == 0, "the slots holding bodies are the low ones"
            nb = bin(have).count("1")
            taken += owner[:nb]
            # every slot's loads address a staged lane's body (an empty slot: the group's first body, one line)
            assert all(o in lanes for o in owner), (hex(m0), owner, have)
            assert owner[nb:] == [owner[0]] * (K_STAGE_BODIES - nb)
        assert taken == lanes, "every staged body is built once, in lane order"
        assert len(groups) == -(-len(lanes) // K_STAGE_BODIES)


def test_staged_moves_partial_groups_rebuild_bodies():
    """Bodies of the chunked workload staged by lanes with gaps in the mask,
    group by group as the schedule hands them out (partial last groups, empty
    slots loading another body's first line): the stores rebuild the oracle's
    bytes."""
    n = 512
    buf, off = rhp.generate(rhp.GEN_CHUNKED, n, 99)
    reqs, _, http, want = run_oracle(buf, off, 16, rhp.MODE_HTTP)
    work = buf.copy()
    bodies = []
    for i in range(n):
        if http["result"][i] != 1 or not http["body_kind"][i]:
            continue
        base, end = int(off[i]) + int(reqs["ret"][i]), int(off[i + 1])
        spans, region = chunk_spans(buf, base, end)
        L = sum(x for _, x in spans)
        if len(spans) > K_MOVE_CHUNKS or (base & 15) + region + 20 > K_STAGE_BODY:
            work[base:base + L] = want[base:base + L]
            continue
        bodies.append((base, spans, region, end - base, int(off[i])))
    rng = np.random.default_rng(3)
    k = 0
    while k < len(bodies):
        # a round of 64 lanes: some lanes staged a body, the others did not
        m = int(rng.integers(1, 1 << 63))
        lanes = [j for j in range(64) if m >> j & 1]
        lane_body = {j: bodies[k + t] for t, j in enumerate(lanes[:len(bodies) - k])}
        m = sum(1 << j for j in lane_body)
        for owner, have in group_schedule(m):
            nb = bin(have).count("1")
            for q in range(K_STAGE_BODIES):   # every slot loads: an empty one the first body's first line
                base = lane_body[owner[q]][0]
                la = base & ~15
                assert 0 <= la and la + 16 <= len(buf)
            stores = [s for q in range(nb) for s in staged_body(buf, *lane_body[owner[q]])]
            for a, v in stores:   # a group's loads land before its stores
                work[a] = v
        k += len(lane_body)
    assert np.array_equal(work, want), f"{int((work != want).sum())} bytes differ from the oracle's"
