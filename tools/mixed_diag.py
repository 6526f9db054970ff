"""Mixed-precision training step error vs the fp32 oracle gradient (host autograd), next to the same step's error
under torch autocast-fp16 / bf16 (the reference's own "16-mixed" arithmetic: the oracle run on the GPU under
torch.autocast), all on the same alignment (the GPU step's MAS path). Usage: python tools/mixed_diag.py [big]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "matcha-tts_amd"), os.path.join(ROOT, "tests"), ROOT):
    sys.path.insert(0, p)
import oracle.matcha_oracle as O  # noqa: E402
import test_gpu_train as T  # noqa: E402
from conftest import HP  # noqa: E402
from matcha_hip.train import MatchaTrainer  # noqa: E402

DEV = "cuda"


def flat_of(g, names):
    return torch.cat([g[n].reshape(-1).double().cpu() for n in names])


def rel(a, b):
    return float((a - b).norm() / b.norm())


def main():
    big = len(sys.argv) > 1 and sys.argv[1] == "big"
    setup = T._configs4_batch() if big else T._setup()
    sd, x, xl, y, yl, t, z = setup
    args = (x.to(DEV), xl.to(DEV), y.to(DEV), yl.to(DEV))
    runs = {}
    for prec in ("32", "16-mixed", "bf16-mixed"):
        tr = MatchaTrainer(sd, HP, DEV, dropout=False, precision=prec)
        out = tr.forward_backward(*args, t=t.to(DEV), z=z.to(DEV))
        S = tr.scaler["scale"] if tr.scaler else 1.0
        runs[prec] = (out["attn"].cpu(), {k: v.detach().cpu() / S for k, v in tr.gradients().items()},
                      [float(out[k]) for k in ("dur_loss", "prior_loss", "cfm_loss")], list(tr.grads.names))
        del tr
    names = runs["32"][3]
    for prec, (attn, g, losses, _) in runs.items():
        (dur, prior, cfm, _, _), gref = T._oracle_grads(sd, x, xl, y, yl, t, z, mas=lambda lp, m, a=attn: a)
        fr = flat_of(gref, names)
        worst = max((rel(g[k].double(), gref[k].double()), k) for k in names
                    if not k.endswith("conv_k.bias") and gref[k].norm() > 0)
        print(f"{prec:11s} attn==fp32run {torch.equal(attn, runs['32'][0])} flat {rel(flat_of(g, names), fr):.3e} "
              f"worst {worst[0]:.3e} {worst[1]} losses rel "
              f"{[abs(a - float(b)) / abs(float(b)) for a, b in zip(losses, (dur, prior, cfm))]}", flush=True)
    # torch autocast on the GPU through the oracle (the reference's 16-mixed arithmetic), same alignment
    attn = runs["32"][0]
    (_, _, _, _, _), gref = T._oracle_grads(sd, x, xl, y, yl, t, z, mas=lambda lp, m: attn)
    fr = flat_of(gref, names)
    for dt in (torch.float16, torch.bfloat16):
        try:
            params = {k: v.clone().float().to(DEV).requires_grad_(True) for k, v in sd.items()
                      if k.startswith(("encoder.", "decoder.estimator."))}
            with torch.autocast("cuda", dtype=dt):
                dur, prior, cfm, _, _ = O.training_losses(params, *(v.to(DEV) for v in (x, xl, y, yl, t, z)), HP,
                                                          mas=lambda lp, m: attn.to(DEV))
                loss = dur + prior + cfm
            grads = torch.autograd.grad(loss * 65536.0 if dt == torch.float16 else loss, list(params.values()),
                                        allow_unused=True)
            s = 1.0 / 65536.0 if dt == torch.float16 else 1.0
            ga = {k: (gr.float().cpu() * s if gr is not None else torch.zeros_like(p).cpu())
                  for (k, p), gr in zip(params.items(), grads)}
            worst = max((rel(ga[k].double(), gref[k].double()), k) for k in names
                        if not k.endswith("conv_k.bias") and gref[k].norm() > 0)
            print(f"autocast {str(dt):15s} flat {rel(flat_of(ga, names), fr):.3e} worst {worst[0]:.3e} {worst[1]}",
                  flush=True)
        except Exception as e:  # report, do not fail the diagnostic
            print(f"autocast {dt} failed: {type(e).__name__}: {str(e)[:200]}", flush=True)


if __name__ == "__main__":
    main()
