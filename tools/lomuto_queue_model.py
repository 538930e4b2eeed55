"""The reference partition (src/index.c:35-47) against the queue model of its ">=" side
(DESIGN.md §3.7 round 5): random ranges of up to 30 rows, outputs compared. Not product code."""
import random
def lomuto(a):
    a=list(a); lo=0; hi=len(a)-1
    piv=a[hi][0]; i=lo-1
    for j in range(lo,hi):
        if a[j][0]<piv:
            i+=1; a[i],a[j]=a[j],a[i]
    a[i+1],a[hi]=a[hi],a[i+1]
    return a, i+1
def model(a):
    n=len(a); hi=n-1; piv=a[hi][0]
    less=[x for x in a[:hi] if x[0]<piv]
    gpos=[k for k in range(hi) if a[k][0]>=piv]
    m=len(gpos); c=len(less)
    if m==0:
        return less+[a[hi]], c
    # insertion positions
    p=[0]*m
    head=None
    for j in range(m):
        if j==0:
            p[0]=0; head=0
        else:
            r=gpos[j]-gpos[j-1]-1
            H=(head+r)%j
            p[j]=H; head=H+1
    rm=(hi-1-gpos[m-1])
    Hf=(head+rm+1)%m if m>1 else 0
    # final list indices by reverse insertion (naive)
    lst=[]
    for j in range(m):
        lst.insert(p[j], j)
    order=[lst[(Hf+t)%m] for t in range(m)]
    out=less+[a[hi]]+[a[gpos[j]] for j in order]
    return out, c
for trial in range(20000):
    n=random.randint(1,30)
    a=[(random.randint(0,random.choice([2,5,50])),k) for k in range(n)]
    x,px=lomuto(a); y,py=model(a)
    assert px==py and x==y, (a,x,y)
print("ok")
