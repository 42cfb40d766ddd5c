"""GPU experiment: A3C config 3 (2^20 boards, CNN bf16) rollout/update time, fused vs torch policy."""
import sys
import torch
sys.path.insert(0, ".")
from rein48_amd.a3c import A3CConfig, A3CTrainer

for fused in (True, False):
    cfg = A3CConfig(n_boards=1 << 20, max_steps=100, mode="textbook", net="cnn", bf16=True, features="exponents",
                    seed=1, update_chunk=10, fused_policy=fused)
    tr = A3CTrainer(cfg, device="cuda:0")
    tr.train_step()
    s = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record(s)
    tr.rollout()
    ev[1].record(s)
    out = tr.update()
    ev[2].record(s)
    torch.cuda.synchronize()
    r, u = ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])
    print("fused=%d rollout %.1f ms (%.2f ms/step, %.1f M env-steps/s)  update %.1f ms  losses %s"
          % (fused, r, r / 100, (1 << 20) * 100 / r / 1e3, u, {k: round(v, 4) for k, v in out.items()}), flush=True)
    del tr
    torch.cuda.empty_cache()
