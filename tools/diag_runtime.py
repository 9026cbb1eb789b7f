"""Diagnose which HIP runtime(s) a process loads when torch and libkompressor_hip are mixed."""
import subprocess, sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SNIPPETS = {
 'torch_first': """
import torch, ctypes
torch.cuda.init(); x = torch.ones(4, device='cuda')
lib = ctypes.CDLL('{root}/kompressor_amd/libkompressor_hip.so')
lib.kmp_last_error.restype = ctypes.c_char_p
print('device_ok', lib.kmp_device_ok(), lib.kmp_last_error())
""",
 'torch_import_first_no_init': """
import torch, ctypes
lib = ctypes.CDLL('{root}/kompressor_amd/libkompressor_hip.so')
lib.kmp_last_error.restype = ctypes.c_char_p
print('device_ok', lib.kmp_device_ok(), lib.kmp_last_error())
x = torch.ones(4, device='cuda'); print('torch ok', x.sum().item())
""",
 'lib_first': """
import ctypes
lib = ctypes.CDLL('{root}/kompressor_amd/libkompressor_hip.so')
lib.kmp_last_error.restype = ctypes.c_char_p
import torch
print('device_ok', lib.kmp_device_ok(), lib.kmp_last_error())
x = torch.ones(4, device='cuda'); print('torch ok', x.sum().item())
""",
}
TAIL = """
maps = open('/proc/self/maps').read().split('\\n')
libs = sorted(set(l.split()[-1] for l in maps if 'amdhip64' in l or 'libhsa-runtime' in l))
print('loaded:', libs)
print('torch hip', torch.version.hip)
"""
for name, code in SNIPPETS.items():
    src = code.format(root=ROOT) + TAIL
    r = subprocess.run([sys.executable, '-c', src], capture_output=True, text=True, timeout=300)
    print('=====', name, 'rc', r.returncode)
    print(r.stdout[-3000:])
    print(r.stderr[-2000:])
