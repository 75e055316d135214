import sys, json
for l in open(sys.argv[1]):
    try: d = json.loads(l)
    except Exception: continue
    if 'kernel' in d and 'us' in d:
        i = d.get('info', {})
        print(f"{d['kernel']:14s} {str(d.get('dtype','')):4s} {str(d.get('cfg','')):9s} us={d['us']:8.1f} GF={d.get('GFLOPs',0):7.1f} frac={d['frac8']:.3f} err={d.get('max_rel_err',0):.2g} S={i.get('slices')} K={i.get('kernel')}")
    else:
        print({k: v for k, v in d.items() if k != 'info'})
