/*
 * Design study (not product, not a test): how many node tests does a closest-
 * hit walk need when it prunes boxes that lie beyond the best hit so far,
 * compared with the reference's exhaustive DFS (hit.c:91-109)? And does the
 * conservative pruning bound ever change a result?
 *
 *   gcc -O2 -ffp-contract=off -fopenmp scripts/prune_study.c -lm -o /tmp/prune_study
 *   /tmp/prune_study [W H nspheres depth rel stack_cap]
 *
 * Walks compared per ray, on the same paths (bounce rays follow the
 * reference's hit, RNG contract mode 1):
 *   dfs     the reference order, no pruning (the oracle's o_bvh_hit)
 *   pdfs    the reference order (left first), prune a box whose entry lower
 *           bound exceeds the best t so far
 *   near    visit the child with the nearer entry first (stack), same pruning
 * Results must be identical: a candidate replaces the best if t < best, or if
 * t == best and it is a later DFS leaf (hit.c:108 ties go right).
 */
#include "../oracle/oracle.c"

#include <stdio.h>

typedef struct {
    double t;
    int sphere, leaf;   /* leaf = DFS (pre-order) number of the leaf node */
    OHit h;
} Best;

static int g_pre;   /* pre-order counter while numbering */
static void number(const ONode *nd);
/* per-node pre-order number cached in the node's count field's neighbour:
   ONode has no spare field, so keep a parallel hash (pointer -> pre) */
#define HBITS 20
static const ONode *hkey[1 << HBITS];
static int hval[1 << HBITS];
static void hput(const ONode *k, int v)
{
    size_t i = ((uintptr_t)k >> 4) & ((1 << HBITS) - 1);
    while (hkey[i]) i = (i + 1) & ((1 << HBITS) - 1);
    hkey[i] = k;
    hval[i] = v;
}
static void number(const ONode *nd)
{
    hput(nd, g_pre++);
    if (nd->first < 0) { number(nd->kid[0]); number(nd->kid[1]); }
}
static int hget(const ONode *k)
{
    size_t i = ((uintptr_t)k >> 4) & ((1 << HBITS) - 1);
    while (hkey[i] != k) i = (i + 1) & ((1 << HBITS) - 1);
    return hval[i];
}

/* Lower bound on the t at which the ray can first be inside the box, in
   double from the float box inflated by `grow` (absolute). */
static double entry_lb(const mirt_ray *r, const mirt_aabb *b, double grow)
{
    const double o[3] = {r->origin.x, r->origin.y, r->origin.z};
    const double d[3] = {r->direction.x, r->direction.y, r->direction.z};
    const double lo[3] = {b->min.x - grow, b->min.y - grow, b->min.z - grow};
    const double hi[3] = {b->max.x + grow, b->max.y + grow, b->max.z + grow};
    double tmin = -INFINITY;
    for (int a = 0; a < 3; a++) {
        if (d[a] == 0.0) {
            if (o[a] < lo[a] || o[a] > hi[a]) return INFINITY;
            continue;
        }
        double t1 = (lo[a] - o[a]) / d[a], t2 = (hi[a] - o[a]) / d[a];
        double n = t1 < t2 ? t1 : t2;
        if (n > tmin) tmin = n;
    }
    return tmin;
}

static double g_rel = 1.0 / 256;   /* relative slack on the best t */

static int better(float t, int leaf, const Best *b) { return b->sphere < 0 || t < b->t || (t == b->t && leaf > b->leaf); }

static void consider_leaf(const mirt_ray *r, const ONode *nd, const mirt_sphere *s, int ns, Best *b, OCount *cnt)
{
    if (cnt) cnt->spheres++;
    if (nd->first >= ns) return;
    OHit h = o_sphere_hit(r, &s[nd->first], nd->first);
    if (!h.hit) return;
    int leaf = hget(nd);
    if (better(h.t, leaf, b)) { b->t = h.t; b->sphere = nd->first; b->leaf = leaf; b->h = h; }
}

static int prunable(const mirt_ray *r, const ONode *nd, const Best *b)
{
    if (b->sphere < 0) return 0;
    /* the sphere may poke out of its rounded box by an ulp; the computed
       t may undershoot the true one (disc cancellation) -- both absorbed
       by the generous slack of this study */
    double e = entry_lb(r, &nd->box, 1e-3);
    return e > b->t * (1.0 + g_rel) + 1e-3;
}

static void pdfs(const mirt_ray *r, const ONode *nd, const mirt_sphere *s, int ns, Best *b, OCount *cnt)
{
    if (cnt) cnt->nodes++;
    if (!o_slab(r, &nd->box)) return;
    if (prunable(r, nd, b)) return;
    if (nd->first >= 0) { consider_leaf(r, nd, s, ns, b, cnt); return; }
    pdfs(r, nd->kid[0], s, ns, b, cnt);
    pdfs(r, nd->kid[1], s, ns, b, cnt);
}

static int g_stack_cap = 128;   /* near-first stack entries; when full, the node's children are walked in DFS order */

static void nearfirst(const mirt_ray *r, const ONode *root, const mirt_sphere *s, int ns, Best *b, OCount *cnt)
{
    const ONode *stack[128];
    int sp = 0;
    if (cnt) cnt->nodes++;
    if (!o_slab(r, &root->box)) return;
    const ONode *nd = root;
    for (;;) {
        if (nd->first >= 0) {
            consider_leaf(r, nd, s, ns, b, cnt);
        } else {
            const ONode *k0 = nd->kid[0], *k1 = nd->kid[1];
            if (cnt) cnt->nodes += 2;
            int h0 = o_slab(r, &k0->box) && !prunable(r, k0, b);
            int h1 = o_slab(r, &k1->box) && !prunable(r, k1, b);
            if (h0 && h1 && sp >= g_stack_cap) {
                /* no room: both subtrees in the reference order, pruned, no stack */
                if (k0->first >= 0) consider_leaf(r, k0, s, ns, b, cnt);
                else { pdfs(r, k0->kid[0], s, ns, b, cnt); pdfs(r, k0->kid[1], s, ns, b, cnt); }
                if (!prunable(r, k1, b)) {
                    if (k1->first >= 0) consider_leaf(r, k1, s, ns, b, cnt);
                    else { pdfs(r, k1->kid[0], s, ns, b, cnt); pdfs(r, k1->kid[1], s, ns, b, cnt); }
                }
            } else if (h0 && h1) {
                double e0 = entry_lb(r, &k0->box, 0), e1 = entry_lb(r, &k1->box, 0);
                if (e1 < e0) { stack[sp++] = k0; nd = k1; } else { stack[sp++] = k1; nd = k0; }
                continue;
            }
            else if (h0) { nd = k0; continue; }
            else if (h1) { nd = k1; continue; }
        }
        for (;;) {
            if (!sp) return;
            nd = stack[--sp];
            if (!prunable(r, nd, b)) break;
        }
    }
}

int main(int argc, char **argv)
{
    int W = argc > 1 ? atoi(argv[1]) : 480, H = argc > 2 ? atoi(argv[2]) : 270;
    int N = argc > 3 ? atoi(argv[3]) : 10000, depth = argc > 4 ? atoi(argv[4]) : 5;
    if (argc > 5) g_rel = atof(argv[5]);
    if (argc > 6) g_stack_cap = atoi(argv[6]);
    mirt_sphere *s = malloc(sizeof(mirt_sphere) * (N + 1));
    o_gen_render_scene(1, N, s);
    ONode *root = o_build(s, 0, N, 0);
    number(root);
    mirt_camera cam;   /* main.c:203-211 */
    memset(&cam, 0, sizeof cam);
    cam.position = v3(0.0f, 4.0f, 50.0f);
    cam.forward = v3(0.0f, 0.0f, -1.0f);
    cam.right = v3(1.0f, 0.0f, 0.0f);
    cam.up = v3(0.0f, 1.0f, 0.0f);
    cam.fov = 45.0f;
    o_mode = 1;
    long long lvl_rays[8] = {0}, n_dfs[8] = {0}, n_p[8] = {0}, n_n[8] = {0}, s_dfs[8] = {0}, s_p[8] = {0}, s_n[8] = {0};
    long long mism = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : mism)
    for (int y = 0; y < H; y++) {
        long long lr[8] = {0}, nd_[8] = {0}, np_[8] = {0}, nn_[8] = {0}, sd[8] = {0}, sp_[8] = {0}, sn[8] = {0};
        for (int x = 0; x < W; x++) {
            mirt_ray ray;
            o_camera_ray_px(&cam, W, H, x, y, &ray);
            o_key = oc_pixel_key(1, (uint32_t)(y * W + x), 0);
            o_draws = 0;
            for (int d = 0; d < depth; d++) {
                OCount c0 = {0, 0}, c1 = {0, 0}, c2 = {0, 0};
                OHit ref = o_bvh_hit(&ray, root, s, N, &c0);
                Best b1 = {0, -1, -1}, b2 = {0, -1, -1};
                pdfs(&ray, root, s, N, &b1, &c1);
                nearfirst(&ray, root, s, N, &b2, &c2);
                int rs = ref.hit ? ref.sphere : -1;
                if (b1.sphere != rs || b2.sphere != rs || (rs >= 0 && (b1.t != ref.t || b2.t != ref.t))) mism++;
                lr[d]++;
                nd_[d] += c0.nodes; np_[d] += c1.nodes; nn_[d] += c2.nodes;
                sd[d] += c0.spheres; sp_[d] += c1.spheres; sn[d] += c2.spheres;
                if (!ref.hit) break;
                V3 dir = o_hemisphere(ref.n);
                ray.origin = ref.p;
                ray.direction = dir;
            }
        }
#pragma omp critical
        for (int d = 0; d < 8; d++) {
            lvl_rays[d] += lr[d]; n_dfs[d] += nd_[d]; n_p[d] += np_[d]; n_n[d] += nn_[d];
            s_dfs[d] += sd[d]; s_p[d] += sp_[d]; s_n[d] += sn[d];
        }
    }
    printf("%dx%d N=%d depth=%d rel=%g mismatches=%lld\n", W, H, N, depth, g_rel, mism);
    printf("level   rays    nodes/ray: dfs  pdfs  near   spheres/ray: dfs  pdfs  near\n");
    for (int d = 0; d < depth; d++) {
        if (!lvl_rays[d]) break;
        double k = (double)lvl_rays[d];
        printf("%5d %8lld   %8.1f %6.1f %6.1f   %8.1f %6.1f %6.1f\n", d, lvl_rays[d], n_dfs[d] / k, n_p[d] / k,
               n_n[d] / k, s_dfs[d] / k, s_p[d] / k, s_n[d] / k);
    }
    return 0;
}

