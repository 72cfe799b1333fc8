"""GPU against the reference's own known-answer vectors, with no hasher of
ours in between.

The reference pins BLAKE3 (hash mode, the mode cas.rs and hash.rs use) with
its Balloon-BLAKE3 vectors: HASH_B3BALLOON_EXPECTED / _WITH_SECRET_EXPECTED
(/root/reference/crates/crypto/src/keys/hashing.rs:180-208, tests :269-321;
balloon-hash 0.4.0, s_cost 131072, t_cost 2).  A Balloon run is 2 752 512
chained BLAKE3 calls on 24-80-byte messages, the output being the digest of
the last one.  The C oracle drives the run (it only concatenates counters and
earlier digests into the next message) and records EVERY message; the GPU
then hashes all of them in one batched K1 call (cas_batch: digest bytes
0..8) and a sample through the tree kernels K2/K3 (checksum_batch_device:
all 32 bytes).  Every GPU digest equals the recorded one, so a Balloon run
driven by the GPU's digests would build the same messages and end on the
same output -- and the last message's 32-byte GPU digest IS the reference's
expected vector, compared with the bytes copied from hashing.rs."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

_S_COST_0 = 131_072


def _transcript(secret: bytes):
    from tests.golden import make_golden as G
    total = _S_COST_0 + G.BALLOON_T_COST * _S_COST_0 * 10  # every BLAKE3 call of the run
    bufs = [np.frombuffer(x if x else b"\0", np.uint8).copy()
            for x in (G.BALLOON_PASSWORD, G.BALLOON_SALT, secret)]
    out = np.zeros(32, np.uint8)
    msg = np.zeros((total, 128), np.uint8)
    ln = np.zeros(total, np.uint32)
    dig = np.zeros((total, 32), np.uint8)
    k = O.lib().orc_balloon_blake3_trace(
        O._ptr(bufs[0]), len(G.BALLOON_PASSWORD), O._ptr(bufs[1]), len(G.BALLOON_SALT),
        O._ptr(bufs[2]), len(secret), _S_COST_0, G.BALLOON_T_COST, O._ptr(out), 1, total,
        O._ptr(msg), O._ptr(ln), O._ptr(dig))
    assert k == total
    return out.tobytes(), msg, ln, dig


@pytest.mark.parametrize("with_secret", [False, True])
def test_gpu_reproduces_reference_balloon_blake3_vector(ctx, with_secret):
    import torch
    from spacedrive_amd import cas, validation
    from tests.golden import make_golden as G
    secret = G.BALLOON_SECRET if with_secret else b""
    expected = (G.BALLOON_WITH_SECRET_EXPECTED if with_secret else G.BALLOON_EXPECTED)[0]
    final, msg, ln, dig = _transcript(secret)
    assert final == expected  # the driver's run is the reference's
    n = ln.size
    assert set(np.unique(ln).tolist()) >= {24, 40, 72}
    off = np.arange(n, dtype=np.uint64) * 128
    # K1 over every message of the run, one batch
    out8, status = cas.cas_batch(msg.reshape(-1), off, ln, ctx=ctx)
    assert not status.any()
    bad = np.flatnonzero(np.any(out8 != dig[:, :8], axis=1))
    assert bad.size == 0, (bad.size, bad[:5])
    # K2/K3 (the full 32 bytes) over a sample and the run's last message
    arena = torch.from_numpy(msg.reshape(-1)).cuda()
    pick = np.unique(np.concatenate([np.arange(0, n, 251), [n - 1]]))
    files = [arena[int(off[i]):int(off[i]) + int(ln[i])] for i in pick]
    out32 = validation.checksum_batch_device(files, ctx=ctx)
    torch.cuda.synchronize()
    got = out32.cpu().numpy()
    np.testing.assert_array_equal(got, dig[pick])
    # the reference's vector, straight from the GPU
    assert bytes(got[-1]) == expected
