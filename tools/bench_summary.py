import json,sys
for f in sys.argv[1:]:
    try:
        l=[x for x in open(f) if x.startswith('{')][-1]; d=json.loads(l)
        r=d['roofline'] or {}
        print(f.split('/')[-1], d['value'], d['ms_per_step'], d['config'].get('contexts_per_gpu'), d['config']['passes_ms'], r.get('frac'), r.get('copy_frac'), d['check'][0]['ok'] if d.get('check') else None)
    except Exception as e:
        print(f, 'ERR', e, open(f).read()[-800:])
