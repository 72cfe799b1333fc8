"""Independent pure-Python BLAKE3 restatement (TEST INFRASTRUCTURE ONLY).

Second, independent restatement of the third-party `blake3` crate 1.4.1 that
`generate_cas_id` (/root/reference/core/src/object/cas.rs:3,24-61) and
`file_checksum` (/root/reference/core/src/object/validation/hash.rs:1,12-21)
call.  The crate is not vendored under /root/reference, so this follows the
published BLAKE3 specification directly.

It is written in the *incremental* style (a chunk state plus a stack of
chaining values merged by the trailing-zero rule), unlike oracle/sd_oracle.c
which builds the tree recursively; agreement between the two on many lengths
pins the tree shape, and both are pinned by the reference's derive_key KAT
(/root/reference/crates/crypto/src/keys/hashing.rs:210-213,324-327).

Pure-Python loops: use for small inputs only (tens of KiB per second).
"""
from __future__ import annotations

import struct

IV = (0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A,
      0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19)
MSG_PERMUTATION = (2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8)

CHUNK_START = 1 << 0
CHUNK_END = 1 << 1
PARENT = 1 << 2
ROOT = 1 << 3
KEYED_HASH = 1 << 4
DERIVE_KEY_CONTEXT = 1 << 5
DERIVE_KEY_MATERIAL = 1 << 6

BLOCK_LEN = 64
CHUNK_LEN = 1024
_M32 = 0xFFFFFFFF


def _rotr(x: int, n: int) -> int:
    return ((x >> n) | (x << (32 - n))) & _M32


def _g(v, a, b, c, d, mx, my):
    v[a] = (v[a] + v[b] + mx) & _M32
    v[d] = _rotr(v[d] ^ v[a], 16)
    v[c] = (v[c] + v[d]) & _M32
    v[b] = _rotr(v[b] ^ v[c], 12)
    v[a] = (v[a] + v[b] + my) & _M32
    v[d] = _rotr(v[d] ^ v[a], 8)
    v[c] = (v[c] + v[d]) & _M32
    v[b] = _rotr(v[b] ^ v[c], 7)


def compress(cv, block_words, counter, block_len, flags):
    """Returns the 16 output words of one compression."""
    v = list(cv) + list(IV[:4]) + [counter & _M32, (counter >> 32) & _M32,
                                   block_len, flags]
    m = list(block_words)
    for rnd in range(7):
        _g(v, 0, 4, 8, 12, m[0], m[1])
        _g(v, 1, 5, 9, 13, m[2], m[3])
        _g(v, 2, 6, 10, 14, m[4], m[5])
        _g(v, 3, 7, 11, 15, m[6], m[7])
        _g(v, 0, 5, 10, 15, m[8], m[9])
        _g(v, 1, 6, 11, 12, m[10], m[11])
        _g(v, 2, 7, 8, 13, m[12], m[13])
        _g(v, 3, 4, 9, 14, m[14], m[15])
        if rnd != 6:
            m = [m[i] for i in MSG_PERMUTATION]
    return [v[i] ^ v[i + 8] for i in range(8)] + [v[i + 8] ^ cv[i] for i in range(8)]


def _words(block: bytes):
    block = block + bytes(BLOCK_LEN - len(block))
    return struct.unpack("<16I", block)


class _Output:
    def __init__(self, cv, words, counter, block_len, flags):
        self.cv, self.words, self.counter = cv, words, counter
        self.block_len, self.flags = block_len, flags

    def chaining_value(self):
        return compress(self.cv, self.words, self.counter, self.block_len, self.flags)[:8]

    def root_bytes(self, n=32):
        out = b""
        ctr = 0
        while len(out) < n:
            w = compress(self.cv, self.words, ctr, self.block_len, self.flags | ROOT)
            out += struct.pack("<16I", *w)
            ctr += 1
        return out[:n]


class _ChunkState:
    def __init__(self, key, chunk_counter, flags):
        self.cv = list(key)
        self.chunk_counter = chunk_counter
        self.flags = flags
        self.block = b""
        self.blocks_compressed = 0

    def length(self):
        return BLOCK_LEN * self.blocks_compressed + len(self.block)

    def _start_flag(self):
        return CHUNK_START if self.blocks_compressed == 0 else 0

    def update(self, data: bytes):
        while data:
            if len(self.block) == BLOCK_LEN:
                self.cv = compress(self.cv, _words(self.block), self.chunk_counter,
                                   BLOCK_LEN, self.flags | self._start_flag())[:8]
                self.blocks_compressed += 1
                self.block = b""
            take = min(BLOCK_LEN - len(self.block), len(data))
            self.block += data[:take]
            data = data[take:]

    def output(self):
        return _Output(self.cv, _words(self.block), self.chunk_counter,
                       len(self.block), self.flags | self._start_flag() | CHUNK_END)


def _parent_output(left_cv, right_cv, key, flags):
    return _Output(key, tuple(left_cv) + tuple(right_cv), 0, BLOCK_LEN, PARENT | flags)


class Hasher:
    """Incremental hasher: update()/finalize(), like blake3::Hasher."""

    def __init__(self, key=IV, flags=0):
        self.key = tuple(key)
        self.flags = flags
        self.chunk = _ChunkState(self.key, 0, flags)
        self.cv_stack = []

    @classmethod
    def new_keyed(cls, key32: bytes):
        return cls(struct.unpack("<8I", key32), KEYED_HASH)

    @classmethod
    def new_derive_key(cls, context: str):
        ctx = cls(IV, DERIVE_KEY_CONTEXT)
        ctx.update(context.encode())
        key = struct.unpack("<8I", ctx.finalize(32))
        return cls(key, DERIVE_KEY_MATERIAL)

    def _add_chunk_cv(self, cv, total_chunks):
        while total_chunks & 1 == 0:
            cv = _parent_output(self.cv_stack.pop(), cv, self.key, self.flags).chaining_value()
            total_chunks >>= 1
        self.cv_stack.append(cv)

    def update(self, data: bytes):
        data = bytes(data)
        while data:
            if self.chunk.length() == CHUNK_LEN:
                cv = self.chunk.output().chaining_value()
                total = self.chunk.chunk_counter + 1
                self._add_chunk_cv(cv, total)
                self.chunk = _ChunkState(self.key, total, self.flags)
            take = min(CHUNK_LEN - self.chunk.length(), len(data))
            self.chunk.update(data[:take])
            data = data[take:]
        return self

    def finalize(self, n=32) -> bytes:
        out = self.chunk.output()
        for cv in reversed(self.cv_stack):
            out = _parent_output(cv, out.chaining_value(), self.key, self.flags)
        return out.root_bytes(n)


def blake3(data: bytes, n: int = 32) -> bytes:
    return Hasher().update(data).finalize(n)


def derive_key(context: str, material: bytes) -> bytes:
    return Hasher.new_derive_key(context).update(material).finalize(32)


def keyed_hash(key32: bytes, data: bytes) -> bytes:
    return Hasher.new_keyed(key32).update(data).finalize(32)


# --- Balloon over BLAKE3 hash mode (the reference's hash-mode KATs) ---

def balloon(pwd: bytes, salt: bytes, secret: bytes, s_cost: int, t_cost: int,
            h=blake3) -> bytes:
    """balloon-hash 0.4.0 Algorithm::Balloon with digest `h` (default: this
    module's BLAKE3), as /root/reference/crates/crypto/src/keys/hashing.rs:95-114
    calls it (p_cost 1; `secret` b"" when the caller passes None, :101).
    Independent of orc_balloon_blake3 in oracle/sd_oracle.c; same algorithm
    (eprint 2016/027 §3.1, delta 3).  Pure Python: small s_cost only unless `h`
    is a fast hash."""
    def u64(x):
        return x.to_bytes(8, "little")
    cnt = 0
    buf = [b""] * s_cost
    buf[0] = h(u64(cnt) + pwd + salt + secret)
    cnt += 1
    for m in range(1, s_cost):
        buf[m] = h(u64(cnt) + buf[m - 1])
        cnt += 1
    for t in range(t_cost):
        for m in range(s_cost):
            buf[m] = h(u64(cnt) + buf[m - 1] + buf[m])  # buf[-1] = buf[s_cost - 1]
            cnt += 1
            for i in range(3):
                idx = h(u64(t) + u64(m) + u64(i))
                other = int.from_bytes(h(u64(cnt) + salt + secret + idx), "little") % s_cost
                cnt += 1
                buf[m] = h(u64(cnt) + buf[m] + buf[other])
                cnt += 1
    return buf[s_cost - 1]


# --- cas.rs restated over in-memory file bytes (independent of the C oracle) ---

SAMPLE_COUNT = 4            # cas.rs:10
SAMPLE_SIZE = 1024 * 10     # cas.rs:11
HEADER_OR_FOOTER_SIZE = 1024 * 8  # cas.rs:12
MINIMUM_FILE_SIZE = 1024 * 100    # cas.rs:15


def cas_id_of_file_bytes(file: bytes, size: int | None = None) -> str:
    """generate_cas_id(path, size) over a file whose bytes are `file`."""
    if size is None:
        size = len(file)
    h = Hasher()
    h.update(size.to_bytes(8, "little"))
    if size <= MINIMUM_FILE_SIZE:
        h.update(file)
    else:
        h.update(file[:HEADER_OR_FOOTER_SIZE])
        jump = (size - 2 * HEADER_OR_FOOTER_SIZE) // SAMPLE_COUNT
        for k in range(SAMPLE_COUNT):
            o = HEADER_OR_FOOTER_SIZE + k * jump
            h.update(file[o:o + SAMPLE_SIZE])
        h.update(file[len(file) - HEADER_OR_FOOTER_SIZE:])
    return h.finalize().hex()[:16]
