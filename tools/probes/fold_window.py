"""Probe (CPU, oracle): distance in ulps between the left-fold running sums of the
SFR scores / squared deviations and the correctly rounded exact prefix sums."""
import sys, math, numpy as np
sys.path[:0]=['/root/repo','/root/repo/metabodecon-rust_amd']
import oracle
from tests.golden.cases import load_case
from fractions import Fraction
def ulps(a, b):
    ia = np.float64(a).view(np.int64); ib = np.float64(b).view(np.int64)
    return int(ia) - int(ib)
for name in ['blood_01','blood_05','synth_128k_2k_s0','sim_03']:
    x,y,sb,st,ign = load_case(name)
    o = oracle.deconvolute(x,y,sb,st,ignore=ign)
    # recompute SFR scores from oracle internals: use sfr via detect+score
    sm = oracle.moving_average(y, 3, 3)
    sd = oracle.second_derivative(sm)
    L,C,R = oracle.detect_peaks(sd)
    absd = np.abs(sd)
    scores = np.array([oracle.score_minimum_sum(absd, int(l), int(c), int(r)) for l,c,r in zip(L,C,R)])
    centers=C
    left,right = oracle.peak_region_boundaries(centers, o.sbi)
    sfr = np.concatenate([scores[:left], scores[right:]])
    for label, t in [('mean', sfr)]:
        acc = -0.0; exact = Fraction(0); worst = 0; devs=[]
        for k, v in enumerate(t):
            acc = acc + float(v); exact += Fraction(float(v))
            d = abs(ulps(acc, float(exact)))
            devs.append(d)
        mean = acc / len(t)
        dev = (sfr - mean)**2
        acc2 = -0.0; exact2 = Fraction(0); devs2=[]
        for v in dev:
            acc2 = acc2 + float(v); exact2 += Fraction(float(v)); devs2.append(abs(ulps(acc2, float(exact2))))
        print(name, 'n_sfr', len(t), 'mean-fold max dev ulps', max(devs), 'p99', np.percentile(devs,99), '| var-fold max', max(devs2), 'p99', np.percentile(devs2,99))
