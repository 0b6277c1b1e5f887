"""Probe (CPU, oracle): do segment chains of the moving average started from the
exact window sum converge to the true running sum? usage: smoother_speculation.py blood_01 synth0"""
import sys, numpy as np
sys.path[:0]=['/root/repo','/root/repo/metabodecon-rust_amd']
import metabodecon as md, oracle
from tests.golden.cases import synth_spectrum

def passes(y, iters=3, ws=3):
    out=[y.copy()]
    v=y.copy()
    for it in range(iters):
        v=oracle.moving_average(v,1,ws); out.append(v.copy())
    return out

def true_sums(v, ws=3):
    # reproduce running sum states (steady state only), index i -> sum after tick i
    right=ws//2; n=len(v); s=0.0; S=np.empty(n)
    from collections import deque
    ring=deque()
    for k in range(right): ring.append(v[k]); s+=v[k]
    for i in range(n-right):
        x=v[i+right]; s+=x
        if len(ring)==ws: p=ring.popleft(); ring.append(x); s-=p
        else: ring.append(x)
        S[i]=s
    return S

def spec_test(v, S, seg, M, ws=3):
    right=ws//2; n=len(v)
    starts=np.arange(seg, n-right-seg, seg)  # segment starts k*seg
    p0=starts-M
    # guess: left fold of window at p0: v[p0+right-ws+1..p0+right]
    g=np.zeros(len(p0))
    for j in range(ws): g=g+v[p0+right-ws+1+j]
    conv_at=np.full(len(p0), -1)
    s=g
    for t in range(1, M+1):
        i=p0+t
        s=(s+v[i+right])-v[i+right-ws]
        eq=(s==S[i])&(conv_at<0)
        conv_at[eq]=t
    return conv_at

for name in sys.argv[1:]:
    if name.startswith('synth'):
        x,y=synth_spectrum(int(name[5:]))[:2]
    else:
        sp=md.Spectrum.read_bruker(f'/root/repo/tests/golden/bruker/blood/{name}',10,10,(-2.2,11.8))
        y=sp.intensities
    P=passes(np.asarray(y,dtype=np.float64))
    for it in range(3):
        v=P[it]; S=true_sums(v)
        c=spec_test(v,S,64,512)
        ok=c>=0
        print(name, 'pass',it, 'unconverged', (~ok).sum(), 'of', len(c), 'conv pct50/90/99/max', np.percentile(c[ok],[50,90,99]), c[ok].max())
