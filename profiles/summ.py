"""One-line summaries of bench.py lines and sac_micro.py JSONs (profiles/gpu_r06.sh)."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    if 'metric' in d:
        s, r, m = d.get('sac') or {}, d['roofline'], d.get('model_fit') or {}
        k = s.get('mlp_kernels') or {}
        print(f, 'value %.1f M/s' % (d['value'] / 1e6), 'roll frac %.4f (%.1f us)' % (r['frac'], r['avg_launch_ms'] * 1e3),
              'sac %.2f TF' % (s.get('achieved_tflops_per_gpu') or 0), 'fit %.4f ms' % (m.get('ms_per_fit_step') or 0),
              ' '.join('%s %.3f/%.1fus' % (n, v['frac'], v['avg_launch_us']) for n, v in k.items()))
    else:
        print(f, 'ms/update %.4f' % d['_total']['ms_per_update'])
        for n, v in sorted(d.items()):
            if ':' in n:
                print('   %-22s %7.2f us %6.2f TF x%d' % (n, v['avg_ms'] * 1e3, v['tflops'], v['launches']))
