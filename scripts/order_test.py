import sys, os
sys.path.insert(0, 'cassandra-accord_amd'); sys.path.insert(0, 'oracle')
mode = sys.argv[1]
if mode == "lib_first":
    from accord_deps import native
    native.lib()
import torch
from accord_deps import native, synth
print("torch", torch.__version__, torch.cuda.is_available())
x = torch.ones(10, device="cuda"); print("torch tensor ok", x.sum().item())
w = synth.random_small(3)
import pyoracle
try:
    got = native.resolve(w); exp = pyoracle.resolve(w); print(mode, "resolve ok equal=", got.equals(exp))
except Exception as e:
    print(mode, "FAILED", e)
import re
maps = open('/proc/self/maps').read()
print(sorted(set(re.findall(r'\S*libamdhip64\S*', maps))))
print(sorted(set(re.findall(r'\S*libhsa-runtime\S*', maps))))
