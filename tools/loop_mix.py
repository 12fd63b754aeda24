"""Instruction mix of the loop that follows an asm marker in a gfx950 .s file.

usage: python tools/loop_mix.py file.s <kernel-name-regex> <marker>
(build with hipcc --cuda-device-only -S -DGS_ASM_MARKERS)."""
import collections
import re
import sys


def main():
    path, kpat, mk = sys.argv[1:4]
    s = open(path).read().split('\n')
    st = [i for i, l in enumerate(s) if re.match(r'^\S*' + kpat + r'\S*:', l)][0]
    en = [i for i in range(st, len(s)) if s[i].strip().startswith('s_endpgm')][0]
    body = s[st:en]
    mi = [i for i, l in enumerate(body) if mk in l][0]
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r'^(\.LBB\S+):', l)
        if m:
            labels[m.group(1)] = i
    a = b = None
    for i in range(mi, len(body)):
        m = re.search(r's_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)', body[i])
        if m:
            t = m.group(1) or m.group(2)
            if t in labels and mi - 5 <= labels[t] < i:
                a, b = labels[t], i
                break
    c = collections.Counter()
    for l in body[a:b + 1]:
        x = l.strip()
        if not x or x.startswith(('.', ';')) or x.endswith(':'):
            continue
        c[x.split()[0]] += 1
    print(f"loop body lines {a}-{b}: {sum(c.values())} instructions")
    for k, v in c.most_common(30):
        print(f"  {v:4d} {k}")


if __name__ == "__main__":
    main()
