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
    slots, words = _const(text, "kPkSlots"), _const(text, "kPkWords")
    assert "constexpr uint32_t kPkCap = kPkWords - 3;" in text
    cap = words - 3
    # a power-of-two table probed with odd steps: every step is coprime
    assert slots & (slots - 1) == 0
    assert "sst[j] = ((q[j].x << 3) | 8u) & 0xFFF8u;" in text
    steps = {((x << 3) | 8) & 0xFFF8 for x in range(1 << 13)}
    assert all((s // 8) % 2 == 1 and 0 < s < slots * 8 for s in steps)
    # byte offsets wrap at 16 bits: exactly the table
    assert "static_cast<uint16_t>(sa[j] + (hit ? 0u : sst[j]))" in text and slots * 8 == 1 << 16
    assert "sa[j] = live[j] ? (q[j].x >> 16) & 0xFFF8u : threadIdx.x << 3;" in text
    # load: the largest bucket held in LDS against the table
    assert cap / slots <= 0.55
    # the word's index field (12 bits, index + 1, bits 20..31) holds every record
    assert cap + 1 <= 0xFFF + 1
    # table + word area = half of the CU's 160 KiB (two workgroups per CU)
    assert slots * 8 + words * 4 == 160 * 1024 // 2


def test_small_table_steps_are_coprime_with_its_slots():
    text = open(SRC).read()
    slots = _const(text, "kLdsSlots")
    assert "return 1u + 6u * (static_cast<uint32_t>(h) & 1023u);" in text
    steps = {1 + 6 * x for x in range(1024)}
    assert all(math.gcd(s, slots) == 1 and 0 < s < slots for s in steps)
