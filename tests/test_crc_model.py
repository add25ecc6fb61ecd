"""CPU model of the gfx950 CRC32C segment kernel's decomposition (csrc/kernels/crc32c.hip).

The GPU tests check the kernel's results against the host CRC32C; this test
checks, without a GPU, the algebra and data movement the kernel relies on, step
by step as the kernel does them:

* the load layout (load i = 4 * block + j: lane m + 16 r takes word r of piece
  16 j + m of the block) followed by the in-register row transpose with the
  v_permlane16_swap / v_permlane32_swap semantics leaves lane l holding piece l;
* a lookup address built by v_perm_b32 from the CRC register and a per-lane
  constant lands on the right entry of the right table in the replicated LDS
  layout (and in the lane's own bank);
* slice-by-4 over each lane's pieces, the shift over the other lanes' bytes,
  the per-lane shift to the chunk end, the XOR fold and the init term give the
  standard CRC32C of every chunk (full segments, a partial last segment and a
  byte tail).
"""

import numpy as np

from distributed_llm_dissemination_amd import _core

POLY = 0x82F63B78
SEG, BLOCK, PIECE = 16384, 4096, 64


def _tables():
    t0 = []
    for b in range(256):
        c = b
        for _ in range(8):
            c = (c >> 1) ^ (POLY if c & 1 else 0)
        t0.append(c)
    T = [t0]
    for _ in range(3):  # T[k][v]: byte v followed by k zero bytes
        T.append([(x >> 8) ^ t0[x & 0xFF] for x in T[-1]])
    return T


T = _tables()


def _perm(s0, s1, sel):
    """v_perm_b32: each result byte picks a byte of {s0 (bytes 4-7), s1 (bytes 0-3)}, 12 = 0x00."""
    src = [(s1 >> (8 * i)) & 0xFF for i in range(4)] + [(s0 >> (8 * i)) & 0xFF for i in range(4)]
    out = 0
    for k in range(4):
        v = (sel >> (8 * k)) & 0xFF
        out |= (src[v] if v < 8 else 0) << (8 * k)
    return out


def _lds_entry(addr, lane):
    """Decode a byte address of the LDS byte-table layout: two tables per 64 KiB, entry b at row
    b * 256 B, odd table at +128 B, replica r (bank r) at +4 r."""
    pair, b, half, replica = addr >> 16, (addr >> 8) & 0xFF, (addr >> 7) & 1, (addr >> 2) & 31
    assert replica == lane & 31  # the lane reads its own bank: conflict-free
    return T[2 * pair + half][b]


def _step(s, w, lane):
    r = (lane & 31) * 4
    c = [r, 128 + r, 0x10000 + r, 0x10080 + r]  # per table t: (pair << 16) | half * 128 + replica * 4
    s ^= w
    out = 0
    for k in range(4):  # byte k of the word is followed by 3 - k bytes: table 3 - k
        out ^= _lds_entry(_perm(s, c[3 - k], 0x0C020000 | ((4 + k) << 8)), lane)
    return out


def _p16(a, b):
    """v_permlane16_swap: odd rows (16 lanes) of a <-> even rows of b."""
    a, b = a.copy(), b.copy()
    for row in (1, 3):
        a[row * 16:(row + 1) * 16], b[(row - 1) * 16:row * 16] = (b[(row - 1) * 16:row * 16].copy(),
                                                                  a[row * 16:(row + 1) * 16].copy())
    return a, b


def _p32(a, b):
    """v_permlane32_swap: upper half of a <-> lower half of b."""
    a, b = a.copy(), b.copy()
    a[32:], b[:32] = b[:32].copy(), a[32:].copy()
    return a, b


def _row_transpose(r0, r1, r2, r3):
    a0, a1 = _p16(r0, r1)
    b0, b1 = _p16(r2, r3)
    c0, c1 = _p32(a0, b0)
    e0, e1 = _p32(a1, b1)
    return c0, e0, c1, e1  # r0, r1, r2, r3


def _loaded_block(seg, b):
    """The 4 loads of block b: register j, lane m + 16 r holds the 16-B word r of piece 16 j + m."""
    regs = []
    for j in range(4):
        reg = np.zeros((64, 16), dtype=np.uint8)
        for lane in range(64):
            m, r = lane & 15, lane >> 4
            off = b * BLOCK + j * 1024 + PIECE * m + 16 * r
            reg[lane] = seg[off:off + 16]
        regs.append(reg)
    return regs


def _segment_raw(seg, dist_to_chunk_end):
    """Raw CRC of one full 16 KiB segment, shifted to its chunk end (the kernel's wave)."""
    gap = BLOCK - PIECE
    acc = 0
    s = [0] * 64
    for b in range(4):
        regs = _row_transpose(*_loaded_block(seg, b))
        for lane in range(64):
            if b:
                s[lane] = _core.crc32c_shift(s[lane], gap)
            piece = np.concatenate([regs[q][lane] for q in range(4)])
            assert bytes(piece) == bytes(seg[b * BLOCK + PIECE * lane:b * BLOCK + PIECE * (lane + 1)])
            for w in piece.view("<u4"):
                s[lane] = _step(s[lane], int(w), lane)
    for lane in range(64):  # lane l's sub-message ends 64 * (63 - l) bytes before the segment end
        acc ^= _core.crc32c_shift(s[lane], PIECE * (63 - lane) + dist_to_chunk_end)
    return acc


def _partial_raw(seg):
    """A chunk's last, shorter segment: strided 16-B words from a zero register, each shifted to
    the segment end, plus the byte tail."""
    nw = len(seg) // 16
    acc = 0
    for j in range(nw):
        s = 0
        for w in np.frombuffer(bytes(seg[16 * j:16 * j + 16]), dtype="<u4"):
            s = _step(s, int(w), j & 63)
        acc ^= _core.crc32c_shift(s, 16 * (nw - 1 - j))
    for byte in seg[16 * nw:]:
        acc = T[0][(acc ^ int(byte)) & 0xFF] ^ (acc >> 8)
    return acc


def test_row_transpose_hands_lane_l_piece_l():
    regs = [np.arange(64) * 4 + j for j in range(4)]  # register j of lane m+16r: (piece 16j+m, word r)
    out = _row_transpose(*regs)
    for q in range(4):
        for lane in range(64):
            # register q of lane l now holds what register r = l >> 4 held in lane (l & 15) + 16 q
            assert out[q][lane] == regs[lane >> 4][(lane & 15) + 16 * q]


def test_slice_model_matches_crc32c():
    rng = np.random.default_rng(7)
    chunk = 2 * SEG + 4096 + 48 + 5  # two full segments, then a partial one with a byte tail
    data = rng.integers(0, 256, size=chunk, dtype=np.uint8)
    raw = 0
    for k in range(2):
        raw ^= _segment_raw(data[k * SEG:(k + 1) * SEG], chunk - (k + 1) * SEG)
    raw ^= _partial_raw(data[2 * SEG:])
    init_term = _core.crc32c_shift(0xFFFFFFFF, chunk) ^ 0xFFFFFFFF
    assert raw ^ init_term == _core.crc32c(data.tobytes())


def test_fused_unpack_scale_handoff():
    """The fused verify+unpack kernel loads a full segment's scales one segment
    ahead (lane l, register r: scale l + 64 r of the segment) and hands word i of
    lane m + 16 r its scale with ds_bpermute from lane `from`, register base >> 6
    (UnpackVisit::word). Model it for every block size that takes this path: the
    register index is the same for all 64 lanes of a word (one VGPR operand per
    bpermute) and the fetched scale is the word's own, e / BLOCK."""
    for block in (64, 128, 256, 512):
        n_scales = SEG // block
        regs = max(1, n_scales // 64)
        assert regs <= 4  # BLOCK 32 (16 registers) keeps the per-word load
        held = np.full((regs, 64), -1)  # scale index held by (register, lane)
        for r in range(regs):
            for lane in range(64):
                held[r, lane] = lane + 64 * r
        for i in range(16):  # load i = 4 * block4k + j
            base = ((i >> 2) * BLOCK + (i & 3) * 1024) // block
            reg = base >> 6
            assert reg < regs
            for lane in range(64):
                lo = 64 * (lane & 15) + 16 * (lane >> 4)
                frm = (base & 63) + lo // block
                assert 0 <= frm < 64
                e = (i >> 2) * BLOCK + (i & 3) * 1024 + lo  # byte offset of the word in the segment
                assert held[reg, frm] == e // block, (block, i, lane)
                assert (e + 15) // block == e // block  # one scale per 16-B word
