"""Generate the committed golden fixtures in tests/golden/ from oracle/bn254.py.

Run from the repo root:  python3 tests/golden/gen_golden.py
The reference (Rust + un-vendored halo2curves) cannot be built or imported here and ships no BN254
vectors, so these fixtures come from the Python restatement, which is itself
pinned by the reference's Poseidon KATs (Fr), algebraic identities and two independent pairing
formulations (tests/test_oracle_python.py).  Values are hex strings of canonical integers.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import bn254 as b  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def h(x):
    return None if x is None else hex(x)


def hp(pt):
    return None if pt is None else [hex(pt[0]), hex(pt[1])]


def hq(q):
    return None if q is None else [[hex(q[0][0]), hex(q[0][1])], [hex(q[1][0]), hex(q[1][1])]]


def msm_case(name, scalars, bases, store_inputs=True, seeds=None):
    exp = b.native_msm(scalars, bases)
    assert exp == b.pippenger_msm(scalars, bases) == b.pippenger_msm_parallel(scalars, bases, 4)
    c = {"name": name, "n": len(scalars), "expected": hp(exp)}
    if store_inputs:
        c["scalars"] = [h(s) for s in scalars]
        c["bases"] = [hp(p) for p in bases]
    if seeds:
        c["seeds"] = seeds
    return c


def main():
    cases = []
    for n in (1, 2, 3, 63, 64, 65):
        sc = b.gen_scalars(b.SEED_SCALARS, n)
        bs = b.gen_bases(b.SEED_BASES, n)
        cases.append(msm_case(f"random_{n}", sc, bs, seeds={"scalars": b.SEED_SCALARS, "bases": b.SEED_BASES}))
    n = 1023
    sc = b.gen_scalars(b.SEED_SCALARS, n)
    bs = b.gen_bases(b.SEED_BASES, n)
    cases.append(msm_case("random_1023", sc, bs, store_inputs=False,
                          seeds={"scalars": b.SEED_SCALARS, "bases": b.SEED_BASES}))
    bs16 = b.gen_bases(b.SEED_BASES, 16)
    cases.append(msm_case("zero_scalars", [0] * 16, bs16))
    cases.append(msm_case("one_scalars", [1] * 16, bs16))
    cases.append(msm_case("r_minus_1", [b.R - 1] * 16, bs16))
    cases.append(msm_case("powers_of_two", [1 << k for k in range(254)], b.gen_bases(b.SEED_BASES, 254)))
    cases.append(msm_case("repeated_base", b.gen_scalars(7, 33), [b.G1_GEN] * 33))
    cases.append(msm_case("p_and_minus_p", [5, 5, 9, 9], [b.G1_GEN, b.g1_neg(b.G1_GEN), bs16[0], b.g1_neg(bs16[0])]))
    cases.append(msm_case("identity_bases", [3, 4, 5, 6], [None, bs16[1], None, bs16[2]]))
    cases.append(msm_case("all_equal_scalars", [0x1234567890ABCDEF] * 100, b.gen_bases(b.SEED_BASES, 100)))
    cases.append(msm_case("mixed_edges", [0, 1, b.R - 1, 2, 1 << 200, b.R - 2],
                          [bs16[3], bs16[3], bs16[3], None, bs16[4], b.g1_neg(bs16[4])]))
    gens = {
        "scalars": {"seed": hex(b.SEED_SCALARS), "values": [h(s) for s in b.gen_scalars(b.SEED_SCALARS, 8)]},
        "bases": {"seed": hex(b.SEED_BASES), "values": [hp(p) for p in b.gen_bases(b.SEED_BASES, 8)]},
        "bases_start_1000": [hp(p) for p in b.gen_bases(b.SEED_BASES, 4, start=1000)],
    }
    json.dump({"cases": cases, "generator": gens}, open(os.path.join(OUT, "msm.json"), "w"), indent=1)

    dec = []
    g2, sg2, accs = b.gen_decider_case(6, bad=[3])
    accs.append((None, None))
    dec.append({"name": "six_valid_one_bad_plus_identity", "g2": hq(g2), "s_g2": hq(sg2),
                "lhs": [hp(a[0]) for a in accs], "rhs": [hp(a[1]) for a in accs],
                "first_fail": b.decide_all(g2, sg2, accs),
                "gt": [[hex(v) for v in b.f12_to_list(b.decide_gt(g2, sg2, l, r))] for (l, r) in accs]})
    g2b, sg2b, accsb = b.gen_decider_case(4, seed=0xABCDEF)
    dec.append({"name": "all_valid", "g2": hq(g2b), "s_g2": hq(sg2b), "lhs": [hp(a[0]) for a in accsb],
                "rhs": [hp(a[1]) for a in accsb], "first_fail": -1})
    dec.append({"name": "first_bad", "g2": hq(g2b), "s_g2": hq(sg2b),
                "lhs": [hp(b.g1_add(accsb[0][0], b.G1_GEN))] + [hp(a[0]) for a in accsb[1:]],
                "rhs": [hp(a[1]) for a in accsb], "first_fail": 0})
    # swapped lhs/rhs is invalid unless s = 1
    dec.append({"name": "swapped", "g2": hq(g2b), "s_g2": hq(sg2b), "lhs": [hp(accsb[1][1])], "rhs": [hp(accsb[1][0])],
                "first_fail": 0})
    pair = {"e_g1_g2": [hex(v) for v in b.f12_to_list(b.pairing(b.G1_GEN, b.G2_GEN))]}
    acc_r = 0x2F1A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7F8091A2B3C4D5E6F7
    accum = {"r": hex(acc_r), "lhs": [hp(a[0]) for a in accs[:6]], "rhs": [hp(a[1]) for a in accs[:6]]}
    el, er = b.accumulate(accs[:6], acc_r)
    accum["expected"] = [hp(el), hp(er)]
    # KzgAs::create_proof with the challenge from a fresh Poseidon transcript (accumulation.rs:156-176)
    (cl, cr), cr_r, _ = b.create_proof(accs[:6])
    cproof = {"lhs": accum["lhs"], "rhs": accum["rhs"], "r": hex(cr_r), "expected": [hp(cl), hp(cr)]}
    json.dump({"cases": dec, "pairing": pair, "accumulate": accum, "create_proof": cproof},
              open(os.path.join(OUT, "decider.json"), "w"), indent=1)
    # The reference's own known-answer vectors (snark-verifier/src/util/hash/poseidon/tests.rs:6-85)
    kat = {
        "source": "snark-verifier/src/util/hash/poseidon/tests.rs:6-85 (HADES poseidonperm_x5_254_3/_5)",
        "mds_t3": [["7511745149465107256748700652201246547602992235352608707588321460060273774987",
                    "10370080108974718697676803824769673834027675643658433702224577712625900127200",
                    "19705173408229649878903981084052839426532978878058043055305024233888854471533"],
                   ["18732019378264290557468133440468564866454307626475683536618613112504878618481",
                    "20870176810702568768751421378473869562658540583882454726129544628203806653987",
                    "7266061498423634438633389053804536045105766754026813321943009179476902321146"],
                   ["9131299761947733513298312097611845208338517739621853568979632113419485819303",
                    "10595341252162738537912664445405114076324478519622938027420701542910180337937",
                    "11597556804922396090267472882856054602429588299176362916247939723151043581408"]],
        "perm_x5_254_3": {"t": 3, "r_f": 8, "r_p": 57, "input": [0, 1, 2],
                          "output": ["7853200120776062878684798364095072458815029376092732009249414926327459813530",
                                     "7142104613055408817911962100316808866448378443474503659992478482890339429929",
                                     "6549537674122432311777789598043107870002137484850126429160507761192163713804"]},
        "perm_x5_254_5": {"t": 5, "r_f": 8, "r_p": 60, "input": [0, 1, 2, 3, 4],
                          "output": ["18821383157269793795438455681495246036402687001665670618754263018637548127333",
                                     "7817711165059374331357136443537800893307845083525445872661165200086166013245",
                                     "16733335996448830230979566039396561240864200624113062088822991822580465420551",
                                     "6644334865470350789317807668685953492649391266180911382577082600917830417726",
                                     "3372108894677221197912083238087960099443657816445944159266857514496320565191"]},
    }
    json.dump(kat, open(os.path.join(OUT, "poseidon_kat.json"), "w"), indent=1)
    print("fixtures written to", OUT)


if __name__ == "__main__":
    main()
