"""Which host op issues each device launch of one eager TrainStep call
(tools/trainstep_profile.py's model and optimizer): prints, per kernel name,
the launch count per step and the innermost aten ops / Python frames that
issued it.  A study tool for the drop-in training step.

    python tools/studies/launch_origins.py [--config c2] [--kernel direct_copy]
"""
import argparse
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import trainstep_profile as tp  # noqa: E402

import torch  # noqa: E402
import mpvae_step  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(tp.CONFIGS))
    ap.add_argument("--kernel", default="")
    cli = ap.parse_args()
    dev = torch.device("cuda", 0)
    args, model, opt, label, feat = tp.build(cli.config, dev, fused=True)
    ts = mpvae_step.TrainStep(model, opt, args)
    for _ in range(3):
        ts(label, feat)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 with_stack=True) as prof:
        ts(label, feat)
        torch.cuda.synchronize()
    by_kernel = collections.defaultdict(collections.Counter)
    for e in prof.events():
        for k in getattr(e, "kernels", []) or []:
            if cli.kernel and cli.kernel not in k.name:
                continue
            # walk up to the outermost aten op, note the Python frame
            chain, p = [e.name], e.cpu_parent
            while p is not None:
                chain.append(p.name)
                p = p.cpu_parent
            frames = [s for s in (e.stack or []) if "mpvae" in s or "torch/optim" in s
                      or "torch/autograd" in s or "mpvae_step" in s][:3]
            by_kernel[k.name[:90]][" <- ".join(chain[:4]) + " @ " + " | ".join(frames)] += 1
    out = {k: {"launches": sum(c.values()), "origins": c.most_common(12)}
           for k, c in sorted(by_kernel.items(), key=lambda kv: -sum(kv[1].values()))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
