"""Generate kI4Tap (ik_vp8x.hip): libwebp's intra-4 predictors (ik_vp8x.h pred4) as per-pixel taps."""
# tap table of libwebp's ten intra-4 predictors (ik_vp8x.h pred4): per (mode, pixel) the
# op and the indices of its samples in e[] = L K J I X A B C D E F G H
L,K,J,I,X,A,B,C,D,E,F,G,H = range(13)
AVG3, AVG2, COPY, TM, DC = 0, 1, 2, 3, 4
def avg3(a,b,c): return (AVG3, a, b, c)
def avg2(a,b): return (AVG2, a, b, 0)
def cp(a): return (COPY, a, 0, 0)
T = {}
def dst(m, x, y, v): T[(m, x, y)] = v
for y in range(4):
    for x in range(4):
        dst(0, x, y, (DC, 0, 0, 0))
        dst(1, x, y, (TM, [I,J,K,L][y], [A,B,C,D][x], X))
        dst(2, x, y, [avg3(X,A,B), avg3(A,B,C), avg3(B,C,D), avg3(C,D,E)][x])
        dst(3, x, y, [avg3(X,I,J), avg3(I,J,K), avg3(J,K,L), avg3(K,L,L)][y])
m=4
dst(m,0,3,avg3(J,K,L))
for (x,y) in [(0,2),(1,3)]: dst(m,x,y,avg3(I,J,K))
for (x,y) in [(0,1),(1,2),(2,3)]: dst(m,x,y,avg3(X,I,J))
for (x,y) in [(0,0),(1,1),(2,2),(3,3)]: dst(m,x,y,avg3(A,X,I))
for (x,y) in [(1,0),(2,1),(3,2)]: dst(m,x,y,avg3(B,A,X))
for (x,y) in [(2,0),(3,1)]: dst(m,x,y,avg3(C,B,A))
dst(m,3,0,avg3(D,C,B))
m=5
for (x,y) in [(0,0),(1,2)]: dst(m,x,y,avg2(X,A))
for (x,y) in [(1,0),(2,2)]: dst(m,x,y,avg2(A,B))
for (x,y) in [(2,0),(3,2)]: dst(m,x,y,avg2(B,C))
dst(m,3,0,avg2(C,D))
dst(m,0,3,avg3(K,J,I))
dst(m,0,2,avg3(J,I,X))
for (x,y) in [(0,1),(1,3)]: dst(m,x,y,avg3(I,X,A))
for (x,y) in [(1,1),(2,3)]: dst(m,x,y,avg3(X,A,B))
for (x,y) in [(2,1),(3,3)]: dst(m,x,y,avg3(A,B,C))
dst(m,3,1,avg3(B,C,D))
m=6
dst(m,0,0,avg3(A,B,C))
for (x,y) in [(1,0),(0,1)]: dst(m,x,y,avg3(B,C,D))
for (x,y) in [(2,0),(1,1),(0,2)]: dst(m,x,y,avg3(C,D,E))
for (x,y) in [(3,0),(2,1),(1,2),(0,3)]: dst(m,x,y,avg3(D,E,F))
for (x,y) in [(3,1),(2,2),(1,3)]: dst(m,x,y,avg3(E,F,G))
for (x,y) in [(3,2),(2,3)]: dst(m,x,y,avg3(F,G,H))
dst(m,3,3,avg3(G,H,H))
m=7
dst(m,0,0,avg2(A,B))
for (x,y) in [(1,0),(0,2)]: dst(m,x,y,avg2(B,C))
for (x,y) in [(2,0),(1,2)]: dst(m,x,y,avg2(C,D))
for (x,y) in [(3,0),(2,2)]: dst(m,x,y,avg2(D,E))
dst(m,0,1,avg3(A,B,C))
for (x,y) in [(1,1),(0,3)]: dst(m,x,y,avg3(B,C,D))
for (x,y) in [(2,1),(1,3)]: dst(m,x,y,avg3(C,D,E))
for (x,y) in [(3,1),(2,3)]: dst(m,x,y,avg3(D,E,F))
dst(m,3,2,avg3(E,F,G))
dst(m,3,3,avg3(F,G,H))
m=8
for (x,y) in [(0,0),(2,1)]: dst(m,x,y,avg2(I,X))
for (x,y) in [(0,1),(2,2)]: dst(m,x,y,avg2(J,I))
for (x,y) in [(0,2),(2,3)]: dst(m,x,y,avg2(K,J))
dst(m,0,3,avg2(L,K))
dst(m,3,0,avg3(A,B,C))
dst(m,2,0,avg3(X,A,B))
for (x,y) in [(1,0),(3,1)]: dst(m,x,y,avg3(I,X,A))
for (x,y) in [(1,1),(3,2)]: dst(m,x,y,avg3(J,I,X))
for (x,y) in [(1,2),(3,3)]: dst(m,x,y,avg3(K,J,I))
dst(m,1,3,avg3(L,K,J))
m=9
dst(m,0,0,avg2(I,J))
for (x,y) in [(2,0),(0,1)]: dst(m,x,y,avg2(J,K))
for (x,y) in [(2,1),(0,2)]: dst(m,x,y,avg2(K,L))
dst(m,1,0,avg3(I,J,K))
for (x,y) in [(3,0),(1,1)]: dst(m,x,y,avg3(J,K,L))
for (x,y) in [(3,1),(1,2)]: dst(m,x,y,avg3(K,L,L))
for (x,y) in [(3,2),(2,2),(0,3),(1,3),(2,3),(3,3)]: dst(m,x,y,cp(L))
assert len(T) == 160, len(T)
rows = []
for m in range(10):
    vals = []
    for y in range(4):
        for x in range(4):
            op,a,b,c = T[(m,x,y)]
            vals.append(a | (b << 4) | (c << 8) | (op << 12))
    rows.append("    {" + ", ".join(f"0x{v:04x}" for v in vals) + "},")
print("\n".join(rows))
