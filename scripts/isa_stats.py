"""Static instruction mix of a kernel in a device assembly dump (hipcc --cuda-device-only -S).
usage: python scripts/isa_stats.py FILE.s SUBSTRING [--loop]"""
import collections
import re
import sys


def kernels(s):
    return re.findall(r'^(_Z\w+):', s, re.M)


def body(s, name):
    i = s.find(name + ":")
    j = s.find(".Lfunc_end", i)
    return s[i:j]


def stats(text):
    c = collections.Counter()
    for line in text.split('\n'):
        line = line.strip()
        if not line or line.startswith(('.', ';')) or line.endswith(':'):
            continue
        op = line.split()[0]
        if op.startswith(('v_mfma', 'v_smfmac')):
            c['mfma'] += 1
        elif op.startswith('v_'):
            c['valu'] += 1
            c['v:' + op] += 1
        elif op.startswith('ds_read'):
            c['ds_read'] += 1
        elif op.startswith('ds_write'):
            c['ds_write'] += 1
        elif op.startswith(('global_load', 'buffer_load')):
            c['gload'] += 1
        elif op.startswith(('global_store', 'buffer_store')):
            c['gstore'] += 1
        elif op.startswith('s_'):
            c['salu'] += 1
        else:
            c['other:' + op] += 1
    return c


if __name__ == "__main__":
    s = open(sys.argv[1]).read()
    for n in kernels(s):
        if sys.argv[2] in n:
            b = body(s, n)
            c = stats(b)
            top = sorted(((v, k) for k, v in c.items() if k.startswith('v:')), reverse=True)[:25]
            print(n[:140])
            print({k: v for k, v in c.items() if not k.startswith('v:')})
            print(top)
            m = re.search(r'\.vgpr_count:\s+(\d+)', s[s.find(n + ":"):]) 
            break
