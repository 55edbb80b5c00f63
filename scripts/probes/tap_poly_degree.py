"""Max |f32 Horner polynomial - exact ES tap| over the interior taps d = 1..6
of W = 8 for fit degrees 7..10 and three betas (es_tap_poly_fit restated in
numpy). Backs the degree-8 choice of kTapPolyDeg."""
import numpy as np
def fit(beta, deg):
    n=deg+1; out=[]
    for d in range(1,7):
        k=np.arange(n); sk=np.cos(np.pi*(k+0.5)/n)
        x=((sk+1)/2+d)/4-1; f=np.exp(beta*(np.sqrt(1-x*x)-1))
        c=np.polynomial.chebyshev.chebfit(sk,f,deg)
        mono=np.polynomial.chebyshev.cheb2poly(c)
        out.append(mono.astype(np.float32))
    return out
for beta in [2.3*8, 2.1*8, 1.9*8]:
  s=np.linspace(-1,1,200001)
  for deg in [7,8,9,10]:
    m=fit(np.float32(beta),deg); err=0
    for d in range(1,7):
        x=((s+1)/2+d)/4-1; ex=np.exp(beta*(np.sqrt(1-x*x)-1))
        acc=np.zeros_like(s,dtype=np.float32); sf=s.astype(np.float32)
        for c in m[d-1][::-1]: acc=(acc*sf+c).astype(np.float32)
        err=max(err,np.abs(acc-ex).max())
    print(beta,deg,err)
