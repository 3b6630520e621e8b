"""Stem max-pool forward timing (A/B of two libraries via MAUV_LIB): the inference form (f16,
pending BN + ReLU on load, no argmax) and the training form (fp32/bf16 with argmax bytes)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-auv_amd")]
import torch  # noqa: E402

from mauv import ops  # noqa: E402


def run(dt, G, B, H, with_idx):
    C, N = 64, G * B
    dev = "cuda"
    y = torch.randn(N, H, H, C, device=dev).to(dt)
    s, h = torch.rand(G, C, device=dev) + 0.5, torch.randn(G, C, device=dev) * 0.1
    Ho = ops.out_hw(H, 3, 2, 1)
    p = torch.empty(N, Ho, Ho, C, device=dev, dtype=dt)
    idx = torch.empty(N, Ho, Ho, C, device=dev, dtype=torch.uint8) if with_idx else None
    for _ in range(2):
        ops.maxpool_fwd(y, N, H, H, C, p, idx, bn=(s, h, G))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    e0.record()
    for _ in range(reps):
        ops.maxpool_fwd(y, N, H, H, C, p, idx, bn=(s, h, G))
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    nbytes = y.numel() * y.element_size() + p.numel() * p.element_size() + (idx.numel() if with_idx else 0)
    print(f"{str(dt):15s} N={N:5d} {H}x{H} idx={with_idx!s:5s}: {ms:7.3f} ms  "
          f"{nbytes / ms / 1e6:7.0f} GB/s (algorithmic)", flush=True)
    return p, idx


if __name__ == "__main__":
    run(torch.float16, 10, 320, 128, False)
    run(torch.float16, 10, 320, 112, False)
    run(torch.float32, 5, 64, 128, True)
    run(torch.bfloat16, 5, 64, 128, True)
