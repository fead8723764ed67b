"""HBM traffic per launch of one kernel from rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE in separate passes, per /opt/skills/guides/MI355X_MICROARCH.md: units KB,
and gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads -> x2).

usage: python profiles/traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> <kernel-substring> <out.json>
"""
import csv
import json
import os
import sys


def per_dispatch(path, kernel, counter):
    vals = [float(r['Counter_Value']) for r in csv.DictReader(open(path))
            if kernel in r['Kernel_Name'] and r['Counter_Name'] == counter]
    return sum(vals) / len(vals) if vals else None, len(vals)


def main():
    fpath, wpath, kernel, out = sys.argv[1:5]
    f, nf = per_dispatch(fpath, kernel, 'FETCH_SIZE')
    w, nw = per_dispatch(wpath, kernel, 'WRITE_SIZE')
    res = {'kernel': kernel, 'fetch_kb_raw': f, 'write_kb': w, 'dispatches': [nf, nw],
           'fetch_bytes': f * 2 * 1024 if f is not None else None,
           'write_bytes': w * 1024 if w is not None else None}
    res['bytes_per_launch'] = (res['fetch_bytes'] or 0) + (res['write_bytes'] or 0)
    res['note'] = 'FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KB -> bytes, mean per dispatch'
    # the library build these counters describe (bench.py attaches the bytes only to a
    # line measured on the same build)
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    'distributional-reachability-policy-optimization_amd'))
    import build_lib
    res['lib_digest'] = build_lib.source_digest()
    json.dump(res, open(out, 'w'), indent=1)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
