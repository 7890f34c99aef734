import time, sys, math, numpy as np, torch
sys.path.insert(0, '.')
import bench
from expecto_amd import synthetic, beluga
from expecto_amd.genome import DeviceGenome, Fasta
from expecto_amd.pipeline import VariantPipeline, VariantSet, shift_order, to_device
dev = torch.device('cuda', 0)
a = torch.randn(8192, 8192, device=dev)
def busy():
    for _ in range(20): a @ a   # ~ 200+ ms of queued GPU work
torch.cuda.synchronize()
def t(label, fn):
    busy(); t0 = time.perf_counter(); fn(); t1 = time.perf_counter(); torch.cuda.synchronize(); t2 = time.perf_counter()
    print(f"{label}: call {1e3*(t1-t0):.1f} ms, queue drain {1e3*(t2-t1):.1f} ms", flush=True)
t("pin+to", lambda: to_device(np.zeros(1000, np.int64), dev))
t("pin+to again", lambda: to_device(np.zeros(1000, np.int64), dev))
t("torch.empty 1GB", lambda: torch.empty(256 << 20, device=dev))
g = synthetic.genome_bytes(n_contigs=24, contig_len=2_000_000, seed=0)
fa = Fasta.from_dict(g); dg = DeviceGenome(fa)
eng = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=8192).cuda().engine()
eng.set_overflow_check(True)
pipe = VariantPipeline(eng, fa, dg)
snv = synthetic.snvs(g, 2048, seed=3)
vs = VariantSet([s[0] for s in snv], np.array([s[1] for s in snv]), [s[2] for s in snv], [s[3] for s in snv])
sh = shift_order(800)
pipe.predict(vs, sh); torch.cuda.synchronize()
t("prepare", lambda: pipe.prepare(vs, sh))
prep = pipe.prepare(vs, sh); torch.cuda.synchronize()
t("predict(prep)", lambda: pipe.predict(prep))
t("predict(prep) again", lambda: pipe.predict(prep))
y = pipe.predict(prep); torch.cuda.synchronize()
t("diff", lambda: pipe.diff(y))
flag = torch.zeros(1, dtype=torch.int32).pin_memory()
t("overflow_take", lambda: eng.overflow_take(flag))
yh = torch.empty(y.shape, dtype=torch.float32).pin_memory()
t("D2H copy", lambda: yh.copy_(y, non_blocking=True))
t("predict(vs)", lambda: pipe.predict(vs, sh))
