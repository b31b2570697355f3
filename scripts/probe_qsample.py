"""Probe: q_sample kernel vs IEEE fp32 (numpy) element by element."""
import numpy as np
import torch
import sys
sys.path.insert(0, '.')
from diffusion_models_collection_amd import kernels as K
z = np.load('tests/golden/diffusion_ops.npz'); s = np.load('tests/golden/schedules.npz')
a = s['linear/sqrt_alphas_cumprod']; b = s['linear/sqrt_one_minus_alphas_cumprod']
x0 = z['x0']; n = z['noise']; t = z['t']
ref = z['q_sample']
got = K.q_sample(torch.from_numpy(x0).cuda(), torch.from_numpy(n).cuda(), torch.from_numpy(t).cuda(),
                 torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()).cpu().numpy()
tg = (torch.from_numpy(a).cuda()[torch.from_numpy(t).cuda()].view(-1,1,1,1) * torch.from_numpy(x0).cuda() +
      torch.from_numpy(b).cuda()[torch.from_numpy(t).cuda()].view(-1,1,1,1) * torch.from_numpy(n).cuda()).cpu().numpy()
bad = np.nonzero(got != ref)
print('mismatch kernel vs fixture:', len(bad[0]), 'torch-gpu vs fixture:', int((tg != ref).sum()))
for idx in list(zip(*bad))[:5]:
    i = tuple(int(v) for v in idx)
    an = a[t[i[0]]]; bn = b[t[i[0]]]
    print(i, 'x0', x0[i].view(np.uint32), 'n', n[i].view(np.uint32), 'an', an.view(np.uint32), 'bn', bn.view(np.uint32),
          'got', got[i].view(np.uint32), 'ref', ref[i].view(np.uint32), 'u', np.float32(an*x0[i]), 'v', np.float32(bn*n[i]))
