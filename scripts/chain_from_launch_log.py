"""Per-panel critical chain of a DPOTRF run from the GPU manager launch log
(PARSEC_MCA_device_hip_trace_launches=1, stderr): for each panel k the POTRF(k)
group launch->release, the gap to the TRSM(k+1,k) launch, its group, the gap to
the SYRK(k,k+1) launch, its group and the gap to POTRF(k+1), in microseconds.
usage: python scripts/chain_from_launch_log.py launches.log.gz"""
import gzip, re, sys
lines = gzip.open(sys.argv[1], 'rt').read().splitlines()
# last factorization: from the last "L stream 0: POTRF(0)"
start = max(i for i, l in enumerate(lines) if 'L stream 0: POTRF(0)' in l)
lines = lines[start:]
ev = []
for l in lines:
    m = re.match(r'\[engine\] t=(\d+) (\w) (.*)', l)
    if m: ev.append((int(m.group(1)), m.group(2), m.group(3)))
t0 = ev[0][0]
# per panel k: POTRF(k) launch, its R, TRSM group launch with TRSM(k, k+1), its R, SYRK(k,k+1) launch, R, POTRF(k+1) launch
open_groups = {i: [] for i in range(8)}
pl = {}
def note(k, what, t):
    pl.setdefault(k, {})[what] = t - t0
for t, kind, rest in ev:
    if kind == 'L':
        s = int(rest.split(':')[0].split()[-1])
        names = re.findall(r'(\w+)\((\d+)(?:, (\d+))?(?:, (\d+))?\)', rest.split('|')[0])
        open_groups[s].append((t, names))
        for n in names:
            if n[0] == 'POTRF': note(int(n[1]), 'potrf_L', t)
            if n[0] == 'TRSM' and n[2] and int(n[2]) == int(n[1]) + 1: note(int(n[1]), 'trsm_L', t)
            if n[0] == 'SYRK' and n[2] and int(n[2]) == int(n[1]) + 1: note(int(n[1]), 'syrk_L', t)
    elif kind == 'R':
        s = int(rest.split()[1])
        if open_groups[s]:
            tl, names = open_groups[s].pop(0)
            for n in names:
                if n[0] == 'POTRF': note(int(n[1]), 'potrf_R', t)
                if n[0] == 'TRSM' and n[2] and int(n[2]) == int(n[1]) + 1: note(int(n[1]), 'trsm_R', t)
                if n[0] == 'SYRK' and n[2] and int(n[2]) == int(n[1]) + 1: note(int(n[1]), 'syrk_R', t)
print(f"{'k':>3} {'potrf':>7} {'->trsmL':>8} {'trsm':>7} {'->syrkL':>8} {'syrk':>7} {'->potrfL':>9} {'chain':>7}")
for k in sorted(pl):
    p = pl[k]; q = pl.get(k + 1, {})
    try:
        print(f"{k:3d} {p['potrf_R']-p['potrf_L']:7d} {p['trsm_L']-p['potrf_R']:8d} {p['trsm_R']-p['trsm_L']:7d} {p['syrk_L']-p['trsm_R']:8d} {p['syrk_R']-p['syrk_L']:7d} {q.get('potrf_L',0)-p['syrk_R']:9d} {q.get('potrf_L',0)-p['potrf_L']:7d}")
    except KeyError as e:
        print(k, 'missing', e)
