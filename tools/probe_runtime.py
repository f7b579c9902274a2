"""Probe: which HIP runtime our library binds to when torch shares the process."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
order = sys.argv[1]
if order == "torch_first":
    import torch
    torch.zeros(1, device="cuda")
import stringsearchlib_amd as ssl
words, wts, rng = ssl.synth.gen_corpus(2000, seed=1)
gi = ssl.StringIndex(words, 1, wts)
r = gi.score_batch(ssl.synth.gen_queries(words, 1, 10, rng), 0.3, 10)
print(order, "search ok", len(r), r[0][:1])
if order != "torch_first":
    import torch
x = torch.arange(10, device="cuda").sum().item()
print(order, "torch ok", x)
with open("/proc/self/maps") as f:
    libs = sorted({l.split()[-1] for l in f if "amdhip64" in l})
print(order, libs)
