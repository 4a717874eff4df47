"""Instruction census of one kernel in a hipcc -S listing (development aid).

usage: python tools/isa_stats.py listing.s <mangled-name-substring> [--dump A:B]
"""
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    s = open(path).read()
    starts = [i for i in range(len(s)) if s.startswith(pat, i)]
    name_i = next(i for i in starts if s[i - 1] == "\n")
    end = s.index('.Lfunc_end', name_i)
    body = s[name_i:end].split('\n')
    cnt = {}
    for line in body:
        t = line.strip().split(' ')[0]
        if t.startswith(('v_mfma', 's_waitcnt', 'ds_', 'buffer_', 's_barrier', 'global_', 'scratch', 's_sleep')):
            cnt[t] = cnt.get(t, 0) + 1
    print(body[0], len(body), 'lines')
    for k in sorted(cnt):
        print(f'  {k:32s} {cnt[k]}')
    if '--dump' in sys.argv:
        a, b = map(int, sys.argv[sys.argv.index('--dump') + 1].split(':'))
        for k in range(a, min(b, len(body))):
            print(k, body[k])


if __name__ == '__main__':
    main()
