"""Bitwise comparison of two library builds on one training step (same seeds, same inputs):
run `python tools/lib_bitcmp.py save OUT.pt [fp32|bf16]` once per library (MAUV_LIB selects
one; MAUV_CENTRE_Y=0 when the builds centre differently), then `python tools/lib_bitcmp.py
cmp A.pt B.pt`: loss, logits and every gradient tensor equal bit for bit, or the first
differences."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-auv_amd")]
import torch  # noqa: E402


def save(out, dtype):
    import bench
    from mauv.engine import set_precision
    from mauv.models import define_models, DEFAULT_PRIOR
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = define_models(None, 7, DEFAULT_PRIOR)["multimodal_model"].to(dev)
    set_precision(model, torch.bfloat16 if dtype == "bf16" else None)
    B = 16
    x, b, s, y = bench.synthetic_batch(B, 224, 256, dev, 1234)
    model.zero_grad(set_to_none=False)
    logits = model.mc_forward(x, b, s, 3)
    loss = torch.nn.functional.cross_entropy(logits.float().mean(0), y)
    loss.backward()
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().cpu().clone() for n, p in model.named_parameters()
             if p.grad is not None}
    torch.save({"loss": loss.detach().cpu(), "logits": logits.detach().float().cpu(),
                "grads": grads}, out)
    print(f"{dtype}: loss {loss.item():.6f}, {len(grads)} gradient tensors -> {out}")


def cmp(a, b):
    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    bad = [k for k in ("loss", "logits") if not torch.equal(A[k], B[k])]
    for n in A["grads"]:
        if not torch.equal(A["grads"][n], B["grads"][n]):
            bad.append(n)
    print(f"{a} vs {b}: {len(A['grads'])} gradient tensors, loss, logits: "
          + ("bit-identical" if not bad else f"{len(bad)} differ, first {bad[:5]}"))
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "save":
        save(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "bf16")
    else:
        sys.exit(cmp(sys.argv[2], sys.argv[3]))
