import faulthandler, sys, os
faulthandler.enable()
sys.path.insert(0, os.getcwd())
def p(*a): print(*a, flush=True)
p("step0 import torch")
import torch
p("torch", torch.__version__, torch.version.hip, torch.cuda.is_available())
x = torch.ones(4, device="cuda"); p("alloc ok", x.sum().item())
p("step1 load lib")
import ctypes
from spfft_amd.ops._lib import library_path
h = ctypes.CDLL(library_path(), mode=ctypes.RTLD_GLOBAL)
p("loaded")
h.spfft_amd_device_count.restype = ctypes.c_int
p("devcount", h.spfft_amd_device_count())
import spfft_amd as sp
p("step2 grid host")
g = sp.Grid(8,8,8,64, sp.ProcessingUnit.HOST, 1); p("host grid ok")
p("step3 grid gpu")
g = sp.Grid(8,8,8,64, sp.ProcessingUnit.GPU, 1); p("gpu grid ok")
import numpy as np
idx = np.array([(x,y,z) for x in range(8) for y in range(8) for z in range(8)], np.int32)
t = g.create_transform(sp.ProcessingUnit.GPU, sp.TransformType.C2C, 8,8,8,8, idx); p("transform ok")
v = torch.ones(512, dtype=torch.complex128, device="cuda")
out = t.backward(v); torch.cuda.synchronize(); p("backward ok", out.shape, out.abs().max().item())
