#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs of scripts/profile_gpu.sh for the TCSC kernels.
Usage: scripts/pmc_summary.py <prof dir> [kernel_ms]"""
import collections, csv, glob, json, os, sys

d = sys.argv[1]
res = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
for f in sorted(glob.glob(os.path.join(d, 'pmc*/run_counter_collection.csv'))):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        if 'tsg_' not in k:
            continue
        kn = k.split('(')[0].replace('void ', '')
        res[kn][r['Counter_Name']] += float(r['Counter_Value'])
out = {}
for kn, v in res.items():
    o = dict(v)
    cyc = v.get('GRBM_GUI_ACTIVE', 0) / 8  # summed over 8 XCDs
    if cyc:
        for c in ('SQ_INSTS_SALU', 'SQ_INSTS_VALU', 'SQ_INSTS_LDS', 'SQ_INSTS_SMEM'):
            if c in v:
                o[c + '_per_CU_clk'] = v[c] / 256 / cyc
    if 'FETCH_SIZE' in v:
        # gfx950: FETCH_SIZE (KiB) reads 1/2 of a wide coalesced stream's bytes
        # (MI355X_MICROARCH.md HBM section): bytes = 2*FETCH_SIZE*1024
        o['hbm_read_bytes_corrected'] = 2 * v['FETCH_SIZE'] * 1024
    if 'WRITE_SIZE' in v:
        o['hbm_write_bytes'] = v['WRITE_SIZE'] * 1024
    out[kn] = o
json.dump(out, sys.stdout, indent=1)
