import torch
a = torch.rand(8192, 8192, device="cuda") * 2 - 1
b = torch.rand(8192, 8192, device="cuda") * 2 - 1
for _ in range(5):
    c = a @ b
torch.cuda.synchronize()
