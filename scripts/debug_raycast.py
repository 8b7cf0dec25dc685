import sys, torch
sys.path.insert(0, '.')
from parallel_c_programs_amd import ops
gpu = torch.device('cuda')
vol = ops.create_volume(512, background="rand")
reg_cpu, _ = ops.region3d(vol, threshold=1)
reg_gpu, _ = ops.region3d(vol.to(gpu), threshold=1)
reg_gpu = (reg_gpu != 0).to(torch.uint8).cpu()
print("region equal:", torch.equal(reg_cpu, reg_gpu), int(reg_cpu.sum()), int(reg_gpu.sum()))
ref = ops.raycast(vol, reg_cpu, 64)
out = ops.raycast(vol.to(gpu), reg_cpu.to(gpu), 64, method="global").cpu()
d = (ref.int() - out.int())
idx = torch.nonzero(d)
print("sums", int(ref.sum()), int(out.sum()), "ndiff", idx.shape[0])
for i in idx[:20].tolist():
    print(i, int(ref[i[0], i[1]]), int(out[i[0], i[1]]))
