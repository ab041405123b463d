# round-4 GPU job: o / qkv decompositions at 512-2,048 rows (fused epilogues, cold weights)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_pfplan
mkdir -p $O
export TMPDIR=/tmp
V=lib,pf_fused,pp128_fused,pp_fused,pp_mix_fused,pf128_s1_fused,pf128_s2_fused,pf128_s3_fused,pf128_s4_fused,pf256_s1_fused,pf256_s2_fused,pf256_s3_fused,pf256_s4_fused
timeout -k 10 900 python -u tools/prefill_gemm_bench.py --shapes o,qkv --M 512,768,1024,1280,1536,2048 --rounds 3 --cold-mb 1024 --variants $V --out $O/pfplan.jsonl > $O/pfplan.log 2>&1 || { tail -30 $O/pfplan.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r4_pfplan/pfplan.jsonl"):
    d=json.loads(l)
    keys=[k for k in d if k.endswith("fused") or k=="lib"]
    print(d["shape"], d["M"], d["plan"], "best", d["best"], " ".join(f"{k}={d[k]}" for k in keys))
PY
