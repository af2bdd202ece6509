"""Counter-based randomness shared by the torch (autograd / CPU) learner path
and the HIP kernels: Philox4x32-10 on int64 tensors, and the critic's
Dropout(0.2) keep-mask keyed by (seed, call number, global batch row, unit)
exactly as k_critic_grad draws it (csrc/sk_update.hip layer1<true>), so the
two paths train on the same masks and a multi-rank update equals the 1-rank
update on the concatenated batch."""
import torch

_M0, _M1 = 0xD2511F53, 0xCD9E8D57
_W0, _W1 = 0x9E3779B9, 0xBB67AE85
_U32 = 0xFFFFFFFF
# keep iff the word >= ceil(0.2 * 2^32): P(drop) = 0.2 (Dropout(0.2), SkillshotLearner.py:105)
DROP_THRESHOLD = 858993460
DROP_SCALE = 1.25  # Keras inverted dropout: kept units scaled by 1 / (1 - rate)


def _mulhilo(a, c):
    """(hi, lo) 32-bit halves of the 64-bit product of the constant a and the
    uint32 values c (int64 tensor), without int64 overflow."""
    ch, cl = c >> 16, c & 0xFFFF
    p_hi, p_lo = a * ch, a * cl  # < 2^48 each
    mid = p_hi + (p_lo >> 16)
    return mid >> 16, ((mid & 0xFFFF) << 16) | (p_lo & 0xFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 of counters (c0..c3: int64 tensors or ints holding uint32)
    under key (k0, k1); returns 4 int64 tensors of uint32 words."""
    ref = next(t for t in (c0, c1, c2, c3) if torch.is_tensor(t))
    c = [torch.as_tensor(x, dtype=torch.int64, device=ref.device).expand_as(ref) & _U32 for x in (c0, c1, c2, c3)]
    k0, k1 = int(k0) & _U32, int(k1) & _U32
    for _ in range(10):
        hi0, lo0 = _mulhilo(_M0, c[0])
        hi1, lo1 = _mulhilo(_M1, c[2])
        c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
        k0 = (k0 + _W0) & _U32
        k1 = (k1 + _W1) & _U32
    return c


def dropout_keep(seed, call, row0, rows, units=256, device="cpu"):
    """bool [rows, units] keep-mask of global batch rows row0 .. row0 + rows - 1
    (row0 a multiple of 4): word (row & 3) of Philox(((row >> 2), unit,
    call_lo, call_hi); seed) compared with DROP_THRESHOLD."""
    if row0 % 4:
        raise ValueError("row0 must be a multiple of 4")
    r = torch.arange(row0, row0 + rows, dtype=torch.int64, device=device).view(-1, 1)
    u = torch.arange(units, dtype=torch.int64, device=device).view(1, -1)
    grp = (r >> 2).expand(rows, units)
    seed = int(seed)
    if not torch.is_tensor(call):
        call = torch.tensor(int(call), dtype=torch.int64)
    call = call.to(device=device, dtype=torch.int64).reshape(())  # device counter: no host sync, capturable
    w = philox4x32_10(grp, u.expand(rows, units), call & _U32, (call >> 32) & _U32, seed & _U32, (seed >> 32) & _U32)
    words = torch.stack(w, -1)  # [rows, units, 4]
    pick = (r & 3).expand(rows, units).unsqueeze(-1)
    return torch.gather(words, -1, pick).squeeze(-1) >= DROP_THRESHOLD
