"""Scan gfx950 device assembly (hipcc --cuda-device-only -S) for the manual
wait-state hazards that LLVM's hazard recognizer cannot see through inline asm
(MI300/MI355X ISA "manually inserted wait states"), in straight-line code:

  valu_sgpr_vmem  a VALU write of an SGPR (v_readfirstlane, v_readlane, v_cmp
                  into an SGPR pair) read by a VMEM instruction (global_* /
                  buffer_*, incl. LDS-DMA) with < 5 wait states between
  valu_permlane   a VALU write of a VGPR read by v_permlane16/32_swap with < 2
  trans_use       a transcendental (v_exp/log/rcp/sqrt/rsq/sin/cos) result read
                  by a non-transcendental VALU op with < 1
  valu_dpp        a VALU write of a VGPR read through DPP with < 2
  m0_lds_dma      an SALU write of M0 followed by an LDS-DMA with < 1

Only reports a pair when the producer or the consumer sits inside an
;;#ASMSTART/;;#ASMEND block (the compiler pads its own instructions).  A label
between the two ends the window (control may arrive from elsewhere; those
paths are reported separately with the label noted).

    python tools/studies/hazard_scan.py file.s [kernel-substring]
"""
import re
import sys

ALL = False
TRANS = re.compile(r"^v_(exp|log|rcp|rsq|sqrt|sin|cos)_f(16|32)")
REG = re.compile(r"\b([vs])(\d+)\b|\b([vs])\[(\d+):(\d+)\]")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out.add((m.group(1), int(m.group(2))))
        else:
            k, a, b = m.group(3), int(m.group(4)), int(m.group(5))
            out.update((k, i) for i in range(a, b + 1))
    if re.search(r"\bm0\b", text):
        out.add(("m0", 0))
    return out


def parse(lines):
    """[(mnemonic, dst regs, src regs, in_asm, raw, wait_states, is_label)]"""
    ins, in_asm = [], False
    for raw in lines:
        s = raw.split(";")[0].strip() if not raw.strip().startswith(";;#ASM") else raw.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not s or s.startswith("."):
            continue
        if s.endswith(":"):
            ins.append(("<label>", set(), set(), False, s, 0, True))
            continue
        parts = s.split(None, 1)
        mn = parts[0]
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        ws = 1
        if mn == "s_nop":
            ws = int(ops[0], 0) + 1 if ops else 1
        dst, src = set(), set()
        if mn.startswith(("global_load_lds", "buffer_load") ) and "lds" in mn:
            src = regs(",".join(ops)) | {("m0", 0)}
        elif mn.startswith(("global_store", "buffer_store", "ds_write", "s_waitcnt", "s_barrier",
                            "s_setprio", "s_nop", "s_sched", "s_branch", "s_cbranch")):
            src = regs(",".join(ops))
        elif mn.startswith(("v_permlane16_swap", "v_permlane32_swap")):
            dst = regs(",".join(ops[:2]))
            src = set(dst)
        elif ops:
            dst = regs(ops[0])
            src = regs(",".join(ops[1:]))
        ins.append((mn, dst, src, in_asm, s, ws, False))
    return ins


def scan(ins):
    found = []
    for j, (mn, dst, src, asm_j, raw, _, lab) in enumerate(ins):
        if lab:
            continue
        checks = []
        if (mn.startswith("global_") or mn.startswith("buffer_")):
            checks.append(("valu_sgpr_vmem", 5, lambda m, d: m.startswith("v_") and
                           any(r[0] == "s" for r in d), {r for r in src if r[0] == "s"}))
        if "lds" in mn and (mn.startswith("global_load") or mn.startswith("buffer_load")):
            checks.append(("m0_lds_dma", 1, lambda m, d: m.startswith("s_") and ("m0", 0) in d,
                           {("m0", 0)}))
        if mn.startswith(("v_permlane16_swap", "v_permlane32_swap")):
            checks.append(("valu_permlane", 2, lambda m, d: m.startswith("v_"),
                           {r for r in src if r[0] == "v"}))
        if mn.startswith("v_") and not TRANS.match(mn):
            checks.append(("trans_use", 1, lambda m, d: bool(TRANS.match(m)),
                           {r for r in src if r[0] == "v"}))
        if "dpp" in raw or "row_" in raw or "quad_perm" in raw:
            checks.append(("valu_dpp", 2, lambda m, d: m.startswith("v_"),
                           {r for r in src if r[0] == "v"}))
        for name, need, is_prod, reads in checks:
            if not reads:
                continue
            waits, crossed = 0, None
            for i in range(j - 1, max(-1, j - 40), -1):
                pm, pd, _, asm_i, praw, pws, plab = ins[i]
                if plab:
                    crossed = praw
                    continue
                hit = pd & reads
                if hit:
                    if is_prod(pm, pd) and waits < need and (asm_i or asm_j or ALL):
                        found.append((name, waits, need, ins[i][4], raw, crossed))
                    reads = reads - hit
                    if not reads:
                        break
                waits += pws
                if waits >= need:
                    break
    return found


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else None
    lines = open(path).read().splitlines()
    # split per kernel (".globl name" ... next ".globl")
    kernels, cur, name = {}, [], None
    for ln in lines:
        m = re.match(r"\s*\.globl\s+(\S+)", ln)
        if m:
            if name:
                kernels[name] = cur
            name, cur = m.group(1), []
        cur.append(ln)
    if name:
        kernels[name] = cur
    total = 0
    for k, body in kernels.items():
        if want and want not in k:
            continue
        hz = scan(parse(body))
        total += len(hz)
        for name, w, need, prod, cons, crossed in hz:
            print(f"{k[:60]}: {name}: {w}/{need} wait states: [{prod}] -> [{cons}]"
                  + (f" (across {crossed})" if crossed else ""))
    print(f"{total} hazard(s)")


if __name__ == "__main__":
    main()
