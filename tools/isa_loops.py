"""Instruction mix of the step loops of one kernel in a hipcc -S listing.

    python tools/isa_loops.py <file.s> <kernel-symbol-regex> [n_loops]

Finds the function, its backward branches (loops), and prints for the largest
loops the instruction count by class (VALU / MFMA / LDS / VMEM / SALU) and the
most frequent opcodes — the per-step instruction budget DESIGN.md quotes."""
import re
import sys
from collections import Counter


def main():
    path, pat = sys.argv[1], re.compile(sys.argv[2])
    nl = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.endswith(":") is False and re.match(r"^\S+:", l) and pat.search(l.split(":")[0]))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    print(body[0][:150])
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, l in enumerate(body):
        m = re.search(r"s_(?:c)?branch\w*\s+(\.LBB\S+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i))
    # keep outermost-largest distinct loops
    loops.sort(key=lambda x: x[0] - x[1])
    shown = []
    for lo, hi in loops:
        if any(lo >= a and hi <= b for a, b in shown):
            continue
        shown.append((lo, hi))
        if len(shown) > nl:
            break
        cnt = Counter()
        for l in body[lo:hi + 1]:
            l = l.strip()
            if not l or l[0] in ";." or l.endswith(":"):
                continue
            cnt[l.split()[0]] += 1
        cls = Counter()
        for op, n in cnt.items():
            k = ("mfma" if op.startswith("v_mfma") else "lds" if op.startswith("ds_") else
                 "vmem" if op.startswith(("global_", "buffer_", "flat_", "scratch_")) else
                 "salu" if op.startswith("s_") else "valu" if op.startswith("v_") else op)
            cls[k] += n
        print(f"loop lines {lo}-{hi}: {sum(cnt.values())} instructions", dict(cls))
        print("   ", ", ".join(f"{op} {n}" for op, n in cnt.most_common(30)))


if __name__ == "__main__":
    main()
