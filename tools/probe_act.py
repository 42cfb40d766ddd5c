import sys, time, torch
sys.path.insert(0, ".")
from rein48_amd.dqn import DQNConfig, DQNTrainer
from rein48_amd.dqn.fused import pack_resnet, pack_resnet_gpu
cfg = DQNConfig(n_boards=1 << 21, replay_capacity=1 << 25, batch=1 << 16, learn_start=1, seed=1, act_chunk=1 << 18)
tr = DQNTrainer(cfg, device="cuda:0")
tr.train_step()
def t(fn, reps=3):
    torch.cuda.synchronize(); a=torch.cuda.Event(enable_timing=True); b=torch.cuda.Event(enable_timing=True)
    w=time.perf_counter(); a.record()
    for _ in range(reps): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b)/reps, (time.perf_counter()-w)*1e3/reps
def act_after_update():
    tr._version += 1
    tr.act()
print("act cached pack   gpu/wall ms", t(tr.act))
print("act + repack      gpu/wall ms", t(act_after_update))
print("pack (PyTorch)    gpu/wall ms", t(lambda: pack_resnet(tr.net)))
print("pack (HIP)        gpu/wall ms", t(lambda: pack_resnet_gpu(tr.net)))
print("update            gpu/wall ms", t(tr.update))
