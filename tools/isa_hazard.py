"""Static check of gfx950 assembly (hipcc -S) for one hazard class the
compiler does not guard: an inline-asm VALU instruction reading (or
overwriting) a register that an MFMA wrote, without the wait states the
MFMA's result needs.

LLVM's hazard recognizer pads its own instructions, but it does not look
at the operands of an inline-asm statement: an asm `v_min3_f32` right after
the `v_mfma` that writes its source read stale accumulator values
(wrong labels at d = 48, k = 777).  The product avoids that
by reading the accumulator with a compiler-visible instruction first
(`min16`, dkm_b2.h), after which the hazard is already paid.

Rule, for every VGPR/AGPR an asm-block VALU instruction reads or writes:
walk the control flow backwards (fall-through and every branch to a label)
counting wait states (1 per instruction, N + 1 per `s_nop N`); the path is
safe once it reaches MIN_STATES, or a compiler-emitted (non-asm)
instruction that touches the register (the compiler waited for it there);
it is a violation when it reaches the MFMA that wrote the register first
with fewer wait states than that MFMA's result needs (`required`).  A
compiler-emitted read of ANY register of that MFMA's destination on the
path also makes it safe: the compiler waited for the MFMA there, and one
wait covers the whole destination.  Wait states for a VALU access after an
XDL MFMA: 12 for the 8-pass gfx950 shapes (cdna_hip_programming.md
"8-pass XDL: 12 states"), 8 for 4-pass, 20 (the 16-pass figure, the
largest) for any shape not in the table.
"""
import re

MIN_STATES = 20          # search depth: the largest requirement
_PASSES = {"v_mfma_f32_32x32x16_bf16": 8, "v_mfma_f32_32x32x16_f16": 8,
           "v_mfma_f32_16x16x32_bf16": 4, "v_mfma_f32_16x16x32_f16": 4}
_STATES = {2: 6, 4: 8, 8: 12, 16: 20}


def required(op):
    """Wait states a VALU access to the destination of MFMA `op` needs."""
    return _STATES.get(_PASSES.get(op, 16), MIN_STATES)


_REG = re.compile(r"\b([va])(?:(\d+)|\[(\d+):(\d+)\])")
_LABEL = re.compile(r"^(\.?L\w+|[A-Za-z_][\w.$]*):")
_BRANCH = re.compile(r"^\s*s_(?:c?branch\w*|setpc_b64)\s+(\S+)")


def _regs(text):
    out = set()
    for m in _REG.finditer(text):
        kind = m.group(1)
        if m.group(2) is not None:
            out.add((kind, int(m.group(2))))
        else:
            for r in range(int(m.group(3)), int(m.group(4)) + 1):
                out.add((kind, r))
    return out


class _Ins:
    __slots__ = ("op", "args", "asm", "states", "line")

    def __init__(self, op, args, asm, line):
        self.op, self.args, self.asm, self.line = op, args, asm, line
        self.states = 1
        if op == "s_nop":
            try:
                self.states = int(args.split(",")[0].strip(), 0) + 1
            except ValueError:
                self.states = 1


def parse_functions(asm_text):
    """Split assembly into functions: lists of instructions and labels."""
    funcs, cur, in_asm = [], None, False
    for ln, raw in enumerate(asm_text.splitlines(), 1):
        s = raw.split(";", 1)[0] if not raw.lstrip().startswith(";;#ASM") \
            else raw
        st = s.strip()
        if raw.strip().startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if raw.strip().startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not st:
            continue
        if st.startswith(".") and not _LABEL.match(st):
            if st.startswith(".Lfunc_end") or st.startswith(".size"):
                cur = None
            continue
        m = _LABEL.match(st)
        if m:
            name = m.group(1)
            if not name.startswith(".L") and not name.startswith("$"):
                cur = {"name": name, "items": []}
                funcs.append(cur)
            elif cur is not None:
                cur["items"].append(("label", name))
            continue
        if cur is None:
            continue
        parts = st.split(None, 1)
        cur["items"].append(("ins", _Ins(parts[0], parts[1] if len(parts) > 1
                                         else "", in_asm, ln)))
    return funcs


def _mfma_dst(ins):
    if not ins.op.startswith("v_mfma"):
        return set()
    first = ins.args.split(",")[0]
    return _regs(first)


def check_function(fn, min_states=MIN_STATES):
    """Violations in one function: (asm line, register, MFMA line, states)."""
    items = fn["items"]
    label_at = {}
    branches_to = {}
    for i, (kind, v) in enumerate(items):
        if kind == "label":
            label_at[v] = i
        else:
            m = _BRANCH.match(v.op + " " + v.args)
            if m and v.op != "s_setpc_b64":
                branches_to.setdefault(m.group(1), []).append(i)
    out = []

    def preds(i):
        """Indices of instructions that can execute right before item i."""
        res = []
        j = i - 1
        while j >= 0:
            kind, v = items[j]
            if kind == "label":
                for b in branches_to.get(v, []):
                    res.append(b)
                j -= 1
                continue
            if v.op in ("s_branch", "s_endpgm", "s_setpc_b64"):
                return res            # no fall-through into item j + 1
            res.append(j)
            return res
        return res

    for i, (kind, ins) in enumerate(items):
        if kind != "ins" or not ins.asm or not ins.op.startswith("v_") or \
                ins.op.startswith("v_mfma"):
            continue
        for reg in sorted(_regs(ins.args)):
            seen = set()
            stack = [(p, 0, frozenset()) for p in preds(i)]
            while stack:
                j, states, touched = stack.pop()
                if states >= min_states or (j, states, touched) in seen:
                    continue
                seen.add((j, states, touched))
                _, pv = items[j]
                dst = _mfma_dst(pv)
                if reg in dst:
                    if states < required(pv.op) and not (touched & dst):
                        out.append((ins.line, "%s%d" % reg, pv.line, states))
                    continue
                if not pv.asm and not pv.op.startswith("v_mfma"):
                    # (an MFMA taking the register whole as its C operand
                    # needs no wait, so it proves nothing)
                    regs = _regs(pv.args)
                    if reg in regs:
                        continue      # the compiler touched it: it waited
                    touched = touched | frozenset(regs)
                for p in preds(j):
                    stack.append((p, states + pv.states, touched))
    return out


def check_asm(asm_text, min_states=MIN_STATES):
    """All violations in an assembly file, with the function names."""
    bad = []
    for fn in parse_functions(asm_text):
        for v in check_function(fn, min_states):
            bad.append((fn["name"],) + v)
    return bad


if __name__ == "__main__":
    import sys
    for path in sys.argv[1:]:
        res = check_asm(open(path).read())
        print(path, len(res), "violations")
        for r in res[:20]:
            print("  ", r)
