"""List the loops of one kernel in a hipcc -save-temps .s file: for each backward branch,
the loop's instruction count, its vmem loads / stores and every s_waitcnt vmcnt inside
(a vmcnt(0) in a streaming loop drains the prefetch ring).

usage: python tools/isa_loops.py FILE.s KERNEL_SYMBOL"""
import re
import sys


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end") or
               (lines[i].startswith("\t.size") and sym in lines[i]))
    body = lines[start:end]
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    for i, l in enumerate(body):
        m = re.search(r"s_c?branch\w*\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            a = labels[m.group(1)]
            seg = body[a:i + 1]
            ins = [x for x in seg if re.match(r"^\s+[vs]_|^\s+buffer_|^\s+global_|^\s+ds_", x)]
            waits = [re.search(r"vmcnt\((\d+)\)", x).group(1) for x in seg if "vmcnt(" in x]
            nl = sum(1 for x in seg if re.search(r"buffer_load|global_load", x))
            ns = sum(1 for x in seg if re.search(r"buffer_store|global_store", x))
            nexp = sum(1 for x in seg if "v_exp_f32" in x)
            tag = re.sub(r".*; %", "", body[a])[:60]
            print(f"loop {m.group(1)} lines {a}-{i}: {len(ins)} instr, {nl} loads, {ns} stores, {nexp} exp, "
                  f"vmcnt waits {waits} [{tag}]")


if __name__ == "__main__":
    main()
