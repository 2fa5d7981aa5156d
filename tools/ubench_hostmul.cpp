// Host Fq multiply variants (libsvgpu's host Horner / fold arithmetic, csrc/host_ec.hpp) timed as a
// dependent chain on the GPU box's CPU: v1 = host_ec.hpp's f_mul (unsigned __int128 CIOS), v2 =
// unrolled CIOS, v3 = mulx / adcx / adox intrinsics.  Build: clang++ -O3 -I snark-verifier-axiom_amd/csrc
// tools/ubench_hostmul.cpp -o tools/ubench_hostmul (clang: __builtin_subcll) -- use /opt/rocm/lib/llvm/bin/clang++
#include "host_ec.hpp"
#include <chrono>
#include <cstdio>
#include <immintrin.h>
using namespace sv::host;
typedef unsigned long long ull;
// V2: unrolled CIOS, u128, branch-free final subtraction via __builtin_subcll
static inline F mul2(const F& a, const F& b) {
  ull t0=0,t1=0,t2=0,t3=0,t4=0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    ull bi = b.l[i];
    u128 s;
    s = (u128)a.l[0]*bi + t0; t0=(ull)s; ull c=(ull)(s>>64);
    s = (u128)a.l[1]*bi + t1 + c; t1=(ull)s; c=(ull)(s>>64);
    s = (u128)a.l[2]*bi + t2 + c; t2=(ull)s; c=(ull)(s>>64);
    s = (u128)a.l[3]*bi + t3 + c; t3=(ull)s; c=(ull)(s>>64);
    s = (u128)t4 + c; t4=(ull)s; ull t5=(ull)(s>>64);
    ull m = t0 * NP64;
    s = (u128)m*P64[0] + t0; c=(ull)(s>>64);
    s = (u128)m*P64[1] + t1 + c; t0=(ull)s; c=(ull)(s>>64);
    s = (u128)m*P64[2] + t2 + c; t1=(ull)s; c=(ull)(s>>64);
    s = (u128)m*P64[3] + t3 + c; t2=(ull)s; c=(ull)(s>>64);
    s = (u128)t4 + c; t3=(ull)s; t4 = t5 + (ull)(s>>64);
  }
  ull br=0, d0,d1,d2,d3;
  d0 = __builtin_subcll(t0, P64[0], 0, &br);
  d1 = __builtin_subcll(t1, P64[1], br, &br);
  d2 = __builtin_subcll(t2, P64[2], br, &br);
  d3 = __builtin_subcll(t3, P64[3], br, &br);
  ull b2; __builtin_subcll(t4, 0, br, &b2);
  F r; bool ge = !b2;
  r.l[0]=ge?d0:t0; r.l[1]=ge?d1:t1; r.l[2]=ge?d2:t2; r.l[3]=ge?d3:t3;
  return r;
}
// V3: mulx / adcx / adox intrinsics (CIOS, two carry chains)
__attribute__((target("bmi2,adx"))) static inline F mul3(const F& a, const F& b) {
  ull t0=0,t1=0,t2=0,t3=0,t4=0;
  for (int i = 0; i < 4; i++) {
    ull bi = b.l[i], h0,h1,h2,h3, l0,l1,l2,l3;
    l0 = _mulx_u64(a.l[0], bi, &h0);
    l1 = _mulx_u64(a.l[1], bi, &h1);
    l2 = _mulx_u64(a.l[2], bi, &h2);
    l3 = _mulx_u64(a.l[3], bi, &h3);
    unsigned char c1=0, c2=0;
    c1 = _addcarryx_u64(c1, t0, l0, &t0);
    c1 = _addcarryx_u64(c1, t1, h0, &t1);
    c1 = _addcarryx_u64(c1, t2, h1, &t2);
    c1 = _addcarryx_u64(c1, t3, h2, &t3);
    c1 = _addcarryx_u64(c1, t4, h3, &t4);
    ull t5 = c1;
    c2 = _addcarryx_u64(c2, t1, l1, &t1);
    c2 = _addcarryx_u64(c2, t2, l2, &t2);
    c2 = _addcarryx_u64(c2, t3, l3, &t3);
    c2 = _addcarryx_u64(c2, t4, 0, &t4);
    t5 += c2;
    ull m = t0 * NP64, q0,q1,q2,q3,r0,r1,r2,r3, dummy;
    r0 = _mulx_u64(m, P64[0], &q0);
    r1 = _mulx_u64(m, P64[1], &q1);
    r2 = _mulx_u64(m, P64[2], &q2);
    r3 = _mulx_u64(m, P64[3], &q3);
    c1 = 0; c2 = 0;
    c1 = _addcarryx_u64(c1, t0, r0, &dummy);
    c1 = _addcarryx_u64(c1, t1, q0, &t1);
    c1 = _addcarryx_u64(c1, t2, q1, &t2);
    c1 = _addcarryx_u64(c1, t3, q2, &t3);
    c1 = _addcarryx_u64(c1, t4, q3, &t4);
    t5 += c1;
    c2 = _addcarryx_u64(c2, t1, r1, &t1);
    c2 = _addcarryx_u64(c2, t2, r2, &t2);
    c2 = _addcarryx_u64(c2, t3, r3, &t3);
    c2 = _addcarryx_u64(c2, t4, 0, &t4);
    t5 += c2;
    t0=t1; t1=t2; t2=t3; t3=t4; t4=t5;
  }
  ull br=0, d0,d1,d2,d3;
  d0 = __builtin_subcll(t0, P64[0], 0, &br);
  d1 = __builtin_subcll(t1, P64[1], br, &br);
  d2 = __builtin_subcll(t2, P64[2], br, &br);
  d3 = __builtin_subcll(t3, P64[3], br, &br);
  ull b2; __builtin_subcll(t4, 0, br, &b2);
  F r; bool ge = !b2;
  r.l[0]=ge?d0:t0; r.l[1]=ge?d1:t1; r.l[2]=ge?d2:t2; r.l[3]=ge?d3:t3;
  return r;
}
template <class FN> double bench(FN fn, F& out) {
  F a = f_one(); F b = f_add(f_dbl(f_one()), f_one());
  auto t0 = std::chrono::steady_clock::now();
  for (int i=0;i<200000;i++) a = fn(a,b);
  auto t1 = std::chrono::steady_clock::now();
  out = a;
  return std::chrono::duration<double,std::nano>(t1-t0).count()/200000;
}
int main(){
  for (int rep=0; rep<3; rep++) {
    F o1,o2,o3;
    double x1 = bench([](const F&a,const F&b){return f_mul(a,b);}, o1);
    double x2 = bench([](const F&a,const F&b){return mul2(a,b);}, o2);
    double x3 = bench([](const F&a,const F&b){return mul3(a,b);}, o3);
    printf("v1 %.1f  v2 %.1f  v3 %.1f ns  eq %d %d\n", x1, x2, x3, f_eq(o1,o2), f_eq(o1,o3));
  }
  // random check
  F a{{0x1234567890abcdefull, 0xfedcba0987654321ull, 0x1111111111111111ull, 0x0fffffffffffffffull}};
  F b{{0xaaaaaaaaaaaaaaaaull, 0x5555555555555555ull, 0x123456789ull, 0x2fffffffffffffffull}};
  int ok = 1;
  for (int i=0;i<100000;i++){ F x=f_mul(a,b), y=mul2(a,b), z=mul3(a,b); ok &= f_eq(x,y) && f_eq(x,z); a = x; b = f_add(b, x);}
  printf("random ok %d\n", ok);
}
