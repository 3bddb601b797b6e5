"""Per-basic-block instruction mix of one kernel in a device assembly dump (hipcc
--cuda-device-only -S): the blocks that issue MFMAs (the hot loops) with their VALU / LDS /
global counts and branch targets.
usage: python scripts/isa_blocks.py FILE.s SUBSTRING [--all]"""
import collections
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    names = [n for n in re.findall(r'^(_Z\w+):', s, re.M) if sys.argv[2] in n]
    for name in names:
        i = s.find(name + ":")
        j = s.find(".Lfunc_end", i)
        body = s[i:j]
        parts = re.split(r'\n(\.LBB\d+_\d+):', body)
        print(name[:140])
        cur = "entry"
        for k, part in enumerate(parts):
            if k % 2 == 1:
                cur = part
                continue
            c = collections.Counter()
            br = []
            for line in part.split('\n'):
                t = line.strip()
                if not t or t.startswith(('.', ';', '_Z')):
                    continue
                op = t.split()[0]
                if op.startswith(('v_mfma', 'v_smfmac')):
                    c['mfma'] += 1
                elif op.startswith('v_'):
                    c['valu'] += 1
                elif op.startswith('ds_read'):
                    c['dsr'] += 1
                elif op.startswith('ds_write'):
                    c['dsw'] += 1
                elif op.startswith(('global_load', 'buffer_load')):
                    c['gl'] += 1
                elif op.startswith(('global_store', 'buffer_store')):
                    c['gs'] += 1
                elif op.startswith('s_waitcnt'):
                    c['wait'] += 1
                elif op.startswith(('s_cbranch', 's_branch')):
                    br.append(t)
                elif op.startswith('s_'):
                    c['salu'] += 1
            if c.get('mfma') or '--all' in sys.argv:
                print("  %-12s %s %s" % (cur, dict(c), br))


if __name__ == "__main__":
    main()
