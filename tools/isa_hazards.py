"""Wait states the compiler leaves between an MFMA and the instructions that read
its result (the layout-sensitive results).

    python tools/isa_hazards.py listing.s [kernel-regex] [--show N]

For every v_mfma in a hipcc -S listing (gfx950) it finds the later instructions,
up to the next label or branch, that read a register of the MFMA's destination,
and counts the wait states between them (one per instruction, N + 1 for s_nop N).
Prints, per (producer, consumer kind), the minimum distance seen and how often
each distance occurs, so two builds' listings can be compared: a consumer that
a producer's result reaches with fewer wait states than the hardware needs reads
stale accumulators, and the symptom depends on timing (run to run) and on code
layout (which edit moved the instructions).  Consumer kinds: srcC (the MFMA
accumulator input, same opcode or another), srcAB (an MFMA's A / B operand),
valu, lds (ds_* data), mem (global / buffer / scratch store data), other."""
import collections
import re
import sys

REG = re.compile(r"\b([va])(\d+)\b|\b([va])\[(\d+):(\d+)\]")


def regs(op):
    out = set()
    for m in REG.finditer(op):
        if m.group(1):
            out.add((m.group(1), int(m.group(2))))
        else:
            out.update((m.group(3), i) for i in range(int(m.group(4)), int(m.group(5)) + 1))
    return out


def split_ops(rest):
    ops, depth, cur = [], 0, ""
    for ch in rest:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            ops.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        ops.append(cur.strip())
    return ops


NODST = ("ds_write", "ds_store", "global_store", "buffer_store", "scratch_store", "flat_store", "s_", "ds_add",
         "global_atomic", "buffer_atomic")


def parse(path, kre):
    funcs, cur, name = {}, None, None
    for line in open(path):
        m = re.match(r"^([\w.$]+):\s*(;.*)?$", line)
        if m and not m.group(1).startswith(".") and not m.group(1).isdigit():  # (digits: inline-asm local labels)
            name = m.group(1)
            if re.search(kre, name):
                cur = funcs.setdefault(name, [])
            else:
                cur = None
            continue
        if cur is None:
            continue
        if re.match(r"^\.LBB|^\.Ltmp|^\s*\.L|^\d+:", line):
            cur.append(("LABEL", [], set(), set()))
            continue
        s = line.split(";")[0].strip()
        if not s or s.startswith("."):
            continue
        parts = s.split(None, 1)
        opc = parts[0]
        ops = split_ops(parts[1]) if len(parts) > 1 else []
        if opc.startswith(NODST) or opc.startswith("s_"):
            dst, src = set(), set().union(*[regs(o) for o in ops]) if ops else set()
        else:
            dst = regs(ops[0]) if ops else set()
            src = set().union(*[regs(o) for o in ops[1:]]) if len(ops) > 1 else set()
        cur.append((opc, ops, dst, src))
    return funcs


def kind(opc, ops, r):
    if opc.startswith("v_mfma"):
        if len(ops) >= 4 and r & regs(ops[3]):
            return "srcC"
        return "srcAB"
    if opc.startswith("ds_"):
        return "lds"
    if opc.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "mem"
    if opc.startswith("v_"):
        return "valu"
    return "other"


def states(opc, ops):
    if opc == "s_nop":
        return int(ops[0], 0) + 1 if ops else 1
    return 1


VALU_PRODUCERS = "--valu" in sys.argv
CROSS = "--cross-labels" in sys.argv  # follow fall-through into the next block (not branches)


def analyse(funcs, horizon=400):
    hist = collections.defaultdict(collections.Counter)
    examples = collections.defaultdict(list)
    for fname, ins in funcs.items():
        for i, (opc, ops, dst, src) in enumerate(ins):
            # producers: every MFMA; with --valu also every VALU whose result an MFMA reads
            if not dst or not (opc.startswith("v_mfma") or (VALU_PRODUCERS and opc.startswith("v_"))):
                continue
            live, gap = set(dst), 0
            for j in range(i + 1, min(len(ins), i + 1 + horizon)):
                o2, ops2, d2, s2 = ins[j]
                if (o2 == "LABEL" and not CROSS) or o2.startswith(("s_branch", "s_cbranch", "s_setpc", "s_endpgm")):
                    break
                if o2 == "LABEL":
                    continue
                hit = live & s2
                if hit and not opc.startswith("v_mfma") and not o2.startswith("v_mfma"):
                    live -= hit  # (VALU -> non-MFMA consumers: not reported)
                    hit = set()
                if hit:
                    k = kind(o2, ops2, hit)
                    same = o2 == opc
                    key = (opc, k + ("(same opcode)" if k == "srcC" and same else ""), o2 if k in ("srcC", "srcAB") else "")
                    hist[key][gap] += 1
                    if len(examples[(key, gap)]) < 2:
                        examples[(key, gap)].append((fname[:60], ins[i][0] + " " + ", ".join(ins[i][1]),
                                                     o2 + " " + ", ".join(ops2)))
                    live -= hit
                live -= d2
                if not live:
                    break
                gap += states(o2, ops2)
    return hist, examples


def analyse_war(funcs, horizon=400):
    """WAR: an MFMA reads a register as A / B / C; the next instruction that WRITES
    that register, and the wait states between (an XDL op reads its sources over
    its passes)."""
    hist = collections.defaultdict(collections.Counter)
    examples = collections.defaultdict(list)
    for fname, ins in funcs.items():
        for i, (opc, ops, dst, src) in enumerate(ins):
            if not opc.startswith("v_mfma") or len(ops) < 4:
                continue
            roles = {"A": regs(ops[1]), "B": regs(ops[2]), "C": regs(ops[3]) - dst}
            live = {r: k for k, rs in roles.items() for r in rs}
            gap = 0
            for j in range(i + 1, min(len(ins), i + 1 + horizon)):
                o2, ops2, d2, s2 = ins[j]
                if o2 == "LABEL" or o2.startswith(("s_branch", "s_cbranch", "s_setpc", "s_endpgm")):
                    break
                hit = [r for r in d2 if r in live]
                if hit:
                    role = "".join(sorted({live[r] for r in hit}))
                    k = "mfma" if o2.startswith("v_mfma") else kind(o2, ops2, set(hit)) if not o2.startswith(
                        ("ds_read", "global_load", "buffer_load", "scratch_load")) else "load"
                    key = (opc, "src" + role + " overwritten by", k)
                    hist[key][gap] += 1
                    if len(examples[(key, gap)]) < 2:
                        examples[(key, gap)].append((fname[:60], opc + " " + ", ".join(ops), o2 + " " + ", ".join(ops2)))
                    for r in hit:
                        del live[r]
                if not live:
                    break
                gap += states(o2, ops2)
    return hist, examples


def main():
    path = sys.argv[1]
    kre = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "."
    show = int(sys.argv[sys.argv.index("--show") + 1]) if "--show" in sys.argv else 0
    funcs = parse(path, kre)
    hist, ex = analyse_war(funcs) if "--war" in sys.argv else analyse(funcs)
    print(f"{len(funcs)} functions")
    for key in sorted(hist):
        c = hist[key]
        print(f"{key[0]:28s} -> {key[1]:18s} {key[2]:28s} min {min(c):2d}  " +
              " ".join(f"{g}:{n}" for g, n in sorted(c.items())[:8]))
        if show:
            for g in sorted(c)[:show]:
                for e in ex[(key, g)]:
                    print(f"      gap {g}: {e[0]}\n        {e[1]}\n        {e[2]}")


if __name__ == "__main__":
    main()
