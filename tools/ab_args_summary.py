import json,glob,sys,re,collections
d=sys.argv[1]
arms=open(sys.argv[2]).read().splitlines()
res=collections.defaultdict(list)
for f in glob.glob(d+"/a*_r*.json"):
    m=re.search(r"/a(\d+)_r(\d+)\.json",f)
    try: j=json.loads(open(f).read().strip().splitlines()[-1])
    except Exception: continue
    res[int(m.group(1))].append((j["ms_per_step"], j["value"], j["config"]["schedule"]["heavy_pixels_used"]))
for i,a in enumerate(arms,1):
    print(f"{a:40s}", sorted(res[i]))
