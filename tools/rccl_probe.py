import os, torch, torch.distributed as dist
r = int(os.environ["RANK"]); w = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.ones(4, device="cuda") * (r + 1)
dist.all_reduce(x)
print("rank", r, "allreduce", x.tolist(), flush=True)
dist.destroy_process_group()
