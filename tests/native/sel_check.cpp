// Test harness (tests/test_ivox_oracle.py): the device restatement of
// std::nth_element (fast-livo-noted_amd/csrc/stl_select.h) against libstdc++'s
// own std::nth_element on the same arrays — same survivors, same order.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "stl_select.h"

struct DP {  // ivox3d_node.hpp:104-118 DistPoint: compared by dist only
    double dist;
    int idx;
    bool operator<(const DP& r) const { return dist < r.dist; }
};

int main(int argc, char** argv) {
    const int trials = argc > 1 ? std::atoi(argv[1]) : 200000;
    std::mt19937 rng(12345);
    long bad = 0;
    for (int t = 0; t < trials; t++) {
        const int n = 1 + (int)(rng() % (t % 7 == 0 ? 400u : 100u));
        const int levels = 1 + (int)(rng() % 40u);  // few distinct keys: many ties
        std::vector<DP> ref(n);
        std::vector<livo::SelElem> dev(n);
        for (int i = 0; i < n; i++) {
            const float f = (t % 3 == 0) ? (float)(rng() % (unsigned)levels) * 0.125f
                                         : std::ldexp((float)(rng() & 0xFFFFFF), -20);
            ref[i] = DP{(double)f, i};
            dev[i] = livo::SelElem{f, (uint32_t)i};
        }
        if (t % 11 == 0) std::sort(ref.begin(), ref.end()), std::sort(dev.begin(), dev.end(), [](auto& a, auto& b) { return a.d < b.d; });
        if (t % 13 == 0) std::reverse(ref.begin(), ref.end()), std::reverse(dev.begin(), dev.end());
        for (int i = 0; i < n; i++) dev[i].id = (uint32_t)ref[i].idx;
        const int first = (t % 5 == 0 && n > 2) ? (int)(rng() % (unsigned)(n / 2)) : 0;
        const int nth = first + (int)(rng() % (unsigned)(n - first));
        std::nth_element(ref.begin() + first, ref.begin() + nth, ref.end());
        livo::sel_nth_element(dev, first, nth, n);
        for (int i = 0; i < n; i++)
            if ((int)dev[i].id != ref[i].idx || (double)dev[i].d != ref[i].dist) {
                bad++;
                break;
            }
    }
    // Musser's median-of-3 killer (and perturbations of it): exhausts the
    // introselect depth limit, so the __heap_select branch is compared too
    for (int n = 8; n <= 600; n += 2)
        for (int rep = 0; rep < 20; rep++) {
            const int k = n / 2;
            std::vector<int> v(n);
            for (int i = 1; i <= k; i++) {
                if (i % 2) {
                    v[i - 1] = i;
                    v[i] = k + i;
                }
                v[k + i - 1] = 2 * i;
            }
            for (int s = 0; s < rep; s++) std::swap(v[rng() % n], v[rng() % n]);
            std::vector<DP> ref(n);
            std::vector<livo::SelElem> dev(n);
            for (int i = 0; i < n; i++) {
                ref[i] = DP{(double)v[i], i};
                dev[i] = livo::SelElem{(float)v[i], (uint32_t)i};
            }
            const int nth = (int)(rng() % (unsigned)n);
            std::nth_element(ref.begin(), ref.begin() + nth, ref.end());
            livo::sel_nth_element(dev, 0, nth, n);
            for (int i = 0; i < n; i++)
                if ((int)dev[i].id != ref[i].idx) {
                    bad++;
                    break;
                }
        }
    std::printf("%d trials, %ld mismatches\n", trials, bad);
    return bad == 0 ? 0 : 1;
}
