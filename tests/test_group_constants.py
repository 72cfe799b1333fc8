"""The group kernels' open-addressing invariants, read from the kernel source
(csrc/dedup.hip): every double-hashing step must be coprime with its table's
slot count, or a probe sequence cycles through a subset of the slots and a
full enough bucket never finds a free one (the kernel's probe loop has no
other exit).  CPU-only: it checks the constants, the GPU tests check the
groupings."""
import math
import os
import re

SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "spacedrive_amd", "csrc", "dedup.hip")


def _const(text, name):
    m = re.search(rf"constexpr uint32_t {name}\s*=\s*(\d+)", text)
    assert m, name
    return int(m.group(1))


def test_packed_table_steps_are_coprime_with_its_slots():
    text = open(SRC).read()
    slots, cap = _const(text, "kPkSlots"), _const(text, "kPkCap")
    m = re.search(r"__builtin_amdgcn_ubfe\((0x[0-9A-Fa-f]+)u,", text)
    assert m
    nibbles = int(m.group(1), 16)
    assert "step[j] = 30u * (q[j].x & 63u) + 2u * nib + 1u;" in text
    steps = {30 * k + 2 * ((nibbles >> (4 * i)) & 15) + 1 for k in range(64) for i in range(8)}
    assert len(steps) == 512
    assert all(math.gcd(s, slots) == 1 and 0 < s < slots for s in steps)
    # load: the largest bucket held in LDS against the table
    assert cap / slots <= 0.55
    # the word's index field (12 bits, index + 1) holds every record of a bucket
    assert cap + 1 <= 0xFFF + 1


def test_small_table_steps_are_coprime_with_its_slots():
    text = open(SRC).read()
    slots = _const(text, "kLdsSlots")
    assert "return 1u + 6u * (static_cast<uint32_t>(h) & 1023u);" in text
    steps = {1 + 6 * x for x in range(1024)}
    assert all(math.gcd(s, slots) == 1 and 0 < s < slots for s in steps)
