import os, sys, glob, subprocess, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zfec_amd import capi
def place(nums,k):
    slots=[None]*k; sec=iter([n for n in nums if n>=k])
    for n in nums:
        if n<k: slots[n]=n
    return [s if s is not None else next(sec) for s in slots]
d = sys.argv[1]
os.makedirs(d, exist_ok=True)
os.environ["ZFEC_HIP_JIT_CACHE"] = d
for k, m in [(10,16),(20,60)]:
    c = capi.Code(k, m)
    t = time.time(); c.jit_prepare_encode(list(range(k, m))); te = time.time()-t
    t = time.time(); c.jit_prepare_decode(place(list(range(m-k, m)), k)); td = time.time()-t
    print(k, m, "compile enc %.2f dec %.2f" % (te, td))
for f in sorted(glob.glob(d + "/*.co")):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", f], capture_output=True, text=True).stdout
    vals = {}
    for line in out.splitlines():
        line = line.strip()
        for key in (".vgpr_count", ".agpr_count", ".vgpr_spill_count", ".sgpr_count"):
            if line.startswith(key + ":"):
                vals[key[1:]] = line.split(":")[1].strip()
    print(os.path.basename(f)[:40], vals)
