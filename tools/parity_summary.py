"""Summarise the parity errors recorded by the GPU suite (tests/tolerances.py
record, MPVAE_RECORD_ERRS=<jsonl>) into profiles/<round>_parity_errors.json:
per case the largest forward error, the largest gradient error and every
recorded tensor's error.

usage: python tools/parity_summary.py gpurun_out/r3final/parity_errs.jsonl \
           profiles/r03_parity_errors.json "<source note>"
"""
import json
import sys

GRAD_PREFIX = ("d", "grad", "param_")


def is_grad(key):
    return key.startswith(GRAD_PREFIX) and key not in ("delta",)


def main(src, dst, note):
    cases = {}
    for line in open(src):
        rec = json.loads(line)
        errs = rec["errs"]
        # d*_ref_*: the reference's own spread (an fp32 variant of the fp64
        # restatement against it), recorded beside the kernels' errors
        spread = [v for k, v in errs.items() if "_ref_" in k]
        errs_k = {k: v for k, v in errs.items() if "_ref_" not in k}
        fwd = [v for k, v in errs_k.items() if not is_grad(k)]
        grad = [v for k, v in errs_k.items() if is_grad(k)]
        c = cases.setdefault(rec["test"], {"fwd_max": None, "grad_max": None, "errs": {}})
        if fwd:
            c["fwd_max"] = max(fwd + ([c["fwd_max"]] if c["fwd_max"] is not None else []))
        if grad:
            c["grad_max"] = max(grad + ([c["grad_max"]] if c["grad_max"] is not None else []))
        if spread:
            c["ref_spread_max"] = max(spread + [c.get("ref_spread_max", 0.0)])
        for k, v in errs.items():
            c["errs"][k] = max(v, c["errs"].get(k, v))
    out = {"source": note,
           "metric": "normwise max|a-b|/max|b| per output tensor (tests/tolerances.py rel_err); "
                     "fwd_max / grad_max: max over the case's forward / gradient tensors "
                     "(kernel errors; ref_spread_max: the reference's own fp32 spread, keys d*_ref_*) "
                     "(keys d*, grad*, param_* are gradients)",
           "cases": cases}
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    print(f"{len(cases)} cases -> {dst}")


if __name__ == "__main__":
    main(*sys.argv[1:4])
