"""List the loops of each engine kernel that contain slot-group loads (global_load_dwordx4) together
with full vmcnt waits: emission loops whose candidate index is a runtime value. Tool only.
usage: python tools/isa_loops.py /tmp/tg.s   (hipcc --offload-device-only -S output)"""
import re
import sys

s = open(sys.argv[1]).read()
for m in re.finditer(r'^(_ZN\S*(?:tile|misc|cost)_kernel\S*):', s, re.M):
    name = m.group(1)
    i = m.end()
    j = s.index('.Lfunc_end', i)
    body = s[i:j].split('\n')
    labels = {}
    for n, l in enumerate(body):
        mm = re.match(r'^(\.LBB\w+):', l.strip())
        if mm:
            labels[mm.group(1)] = n
    rep = []
    for n, l in enumerate(body):
        mm = re.search(r's_cbranch_\w+\s+(\.LBB\w+)', l) or re.search(r's_branch\s+(\.LBB\w+)', l)
        if mm and mm.group(1) in labels and labels[mm.group(1)] < n:
            a = labels[mm.group(1)]
            seg = body[a:n]
            nx4 = sum('global_load_dwordx4' in x for x in seg)
            nw0 = sum('vmcnt(0)' in x for x in seg)
            nds = sum('ds_write_b64' in x for x in seg)
            if nx4 and nds:
                rep.append(f"  loop {a}-{n}: slot loads {nx4}, vmcnt(0) {nw0}, ds_write_b64 {nds}")
    print(name[:80], f"({len(body)} lines)")
    print("\n".join(rep) if rep else "  no runtime emission loops")
