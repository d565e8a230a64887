set -u
cd $GRAFT_REPO_ROOT
for v in "TDE_BN_MAXCH=256" "TDE_BN_MAXCH=1024 TDE_BN_ELEMS=8192" "TDE_BN_MAXCH=1024 TDE_BN_ELEMS=4096" "TDE_BN_MAXCH=512"; do echo "$v"; env $v timeout -k 10 120 python scripts/layer_profile.py --math bf16x6r --top 300 2>&1 | python3 -c "
import sys
tot={}
for l in sys.stdin:
    p=l.split()
    if len(p)>4 and p[1]=='ms': tot[p[3]]=tot.get(p[3],0)+float(p[0])
    elif l.startswith('total'): print(l.strip())
print({k: round(v,3) for k,v in sorted(tot.items())})" || exit 1
env $v timeout -k 10 200 python bench.py --steps 100 --warmup 20 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'])" || exit 1; done
