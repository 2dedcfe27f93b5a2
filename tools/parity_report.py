"""Parity report (GPU box): fraction of bit-identical outputs and max differences, GPU vs oracle, on
the 8 golden RFMIP columns.  Usage: python tools/parity_report.py"""
import sys, numpy as np, torch
sys.path.insert(0,'rte-rrtmgp-nn_amd'); sys.path.insert(0,'oracle'); sys.path.insert(0,'tests')
from rrtmgpnn import rbin, data
from rrtmgpnn.pipeline import ClearSkyStep
import oracle as O
from conftest import subset
g = rbin.read('tests/golden/rfmip8_reference.rbin')
prob = subset(data.rfmip_problem(), g['cols'])
st = ClearSkyStep(prob, 0); st.step(); torch.cuda.synchronize()
f = st.fluxes()
orc = O.Oracle()
lu, ld, go = orc.clear_sky_lw(prob, [data.load_model('lw_abs'), data.load_model('lw_pfrac')], data.load_kdist('lw'))
su, sd, sr, gs = orc.clear_sky_sw(prob, [data.load_model('sw_abs'), data.load_model('sw_ray')], data.load_kdist('sw'))
for k, r in (('lw_up', lu), ('lw_dn', ld), ('sw_up', su), ('sw_dn', sd), ('sw_dir', sr)):
    a = f[k].copy()
    if k in ('sw_up','sw_dn'): a[~prob['usecol']] = 0
    print(k, 'max abs', np.abs(a-r).max(), 'bitwise frac', np.mean(a==r))
for k in ('tau_lw','lay_src','lev_src','tau_sw','ssa_sw'):
    a = getattr(st, k).cpu().numpy()
    r = {'tau_lw': go['tau'], 'lay_src': go['lay_source'], 'lev_src': go['lev_source'], 'tau_sw': gs['tau'], 'ssa_sw': gs['ssa']}[k]
    print(k, 'bitwise frac', np.mean(a==r), 'max rel', np.max(np.abs(a-r)/np.maximum(np.abs(r),1e-30)))
print('x_lw bitwise', np.mean(st.x_lw.cpu().numpy()==go['nn_inputs']), 'col_dry', np.mean(st.col_dry.cpu().numpy()==go['col_dry']))
