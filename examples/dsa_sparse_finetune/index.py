"""Packed-sequence helpers (reference: examples/dsa_sparse_finetune/index.py).

Sequences of a batch are packed back to back; ``offsets`` [B+1] (int32) are their prefix sums.
``token_indices`` [S, 2] = (sequence id, position in the sequence) per packed token, computed on
the device without a host sync."""


def prepare_token_indices(offsets):
    import torch
    offsets = offsets.to(torch.int64)
    lens = offsets[1:] - offsets[:-1]
    total = int(offsets[-1])
    seq = torch.repeat_interleave(torch.arange(lens.numel(), device=offsets.device), lens, output_size=total)
    pos = torch.arange(total, device=offsets.device) - offsets[:-1][seq]
    return torch.stack([seq, pos], 1).to(torch.int32).contiguous()
