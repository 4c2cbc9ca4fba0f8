/*
 * battle_oracle.c -- TEST ORACLE ONLY.  Single-threaded plain-C restatement of the
 * reference Battle engine (MAgent gridworld as vendored in
 * /root/reference/examples/battle_model/src).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product path never does.
 *
 * Parity: pinned bit-exact against tests/golden/battle_*.npz, which were recorded
 * from the reference engine itself (oracle/_ref, OMP_NUM_THREADS=1) driven through
 * the reference's own python wrapper (tests/golden/make_battle_fixtures.py).
 *
 * It exports the reference C ABI (runtime_api.h:118-181) so the same python driver
 * runs the reference build, this oracle and the HIP engine.  Supported subset = what
 * the Battle path uses: 1x1 agents, NORTH only (turn/food/goal modes
 * off), circle/sector ranges, reward rules on one binary event (attack/kill/collide)
 * between two 'any' symbols; plus can_absorb types (Map.cc:345-364, GridWorld.cc:357-363,
 * :638; pinned against oracle/_ref by tests/test_absorb.py).  Anything else fails loudly
 * (return -1 + stderr).
 *
 * Data layout is its own: agents live in an append-only pool per episode (index =
 * id), groups keep ordered id lists, the map keeps one int per cell
 * (-1 empty, -2 wall, >=0 agent id).
 */
#include <math.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ORC_FAIL(...) do { fprintf(stderr, "battle_oracle: " __VA_ARGS__); fputc('\n', stderr); return -1; } while (0)

enum { OP_AND, OP_OR, OP_NOT, OP_KILL, OP_AT, OP_IN, OP_COLLIDE, OP_ATTACK, OP_DIE,
       OP_IN_A_LINE, OP_ALIGN, OP_NULL };                       /* grid_def.h:17-23 */
#define CELL_EMPTY (-1)
#define CELL_WALL  (-2)
#define MAX_TYPES 8
#define MAX_GROUPS 8
#define MAX_RULES 32
#define MAX_SYM 64

typedef struct {                     /* Range.h:14-113, rectangle + mask + index deltas */
    int w, h, count, x1, y1, x2, y2;
    unsigned char *in;
    int *dx, *dy;
} Range;

typedef struct {                     /* AgentType.h:17-52 (subset) */
    char name[64];
    int width, length;
    float speed, hp, view_radius, view_angle, attack_radius, attack_angle;
    float damage, step_recover, kill_supply, food_supply, eat_ability, trace;
    float hear_radius, speak_radius; int speak_ability;
    bool attack_in_group, can_absorb;
    float step_reward, kill_reward, dead_penalty, attack_penalty;
    int view_x_offset, view_y_offset, att_x_offset, att_y_offset;
    Range view, attack, move;
    int n_action, attack_base, turn_base;
} Type;

typedef struct {                     /* GridWorld.h:134-258 */
    int id, x, y, group, index;
    bool dead, absorbed;             /* absorbed: GridWorld.h:196-197, 238 */
    float hp;
    int last_action, last_op, op_obj; /* op_obj: agent id or -1 */
    float next_reward, last_reward;
} Agent;

typedef struct { int type; int *ids; int n, cap, dead_ct; float reward; } Group;
typedef struct { int id, action, bucket; } Act;
typedef struct { int group, index; } Sym;
typedef struct { int op; int raw[8]; int n_raw; } Node;
typedef struct { int on; int recv[8]; float val[8]; int n_recv; bool terminal; } Rule;

typedef struct {
    int w, h;
    bool minimap_mode, food_mode, turn_mode, goal_mode, large_map_mode;
    int embedding_size, n_sep;
    uint64_t rng;
    Type types[MAX_TYPES]; int n_types;
    Group groups[MAX_GROUPS]; int n_groups;
    int *cells;
    Agent *pool; int n_pool, cap_pool;
    int id_counter;
    Act *atk; int n_atk, cap_atk;
    Act *mov; int n_mov, cap_mov;
    Sym syms[MAX_SYM]; int n_syms;
    Node nodes[MAX_SYM]; int n_nodes;
    Rule rules[MAX_RULES]; int n_rules;
    bool rule_trigger[MAX_RULES];
} Env;

/* ---------------------------------------------------------------- RNG -------- */
/* std::default_random_engine == minstd_rand0 (GridWorld.h:106): x <- 16807 x mod (2^31-1) */
static void rng_seed(Env *e, unsigned long s) { uint64_t x = s % 2147483647UL; e->rng = x ? x : 1; }
static uint64_t rng_next(Env *e) { e->rng = (e->rng * 16807ULL) % 2147483647ULL; return e->rng; }

/* ---------------------------------------------------------------- ranges ----- */
static void range_alloc(Range *r) {
    r->in = calloc((size_t)r->w * r->h, 1);
    r->dx = calloc((size_t)r->w * r->h, sizeof(int));
    r->dy = calloc((size_t)r->w * r->h, sizeof(int));
}
/* CircleRange (Range.h:171-215) */
static void circle_range(Range *r, float radius, float inner, int parity) {
    const double eps = 1e-8;
    int width = 2 * (int)(radius + eps) + parity, center = (int)radius;
    if (width % 2 != parity) width++;
    r->w = r->h = width; range_alloc(r); r->count = 0;
    double delta = parity == 0 ? 0.5 : 0;
    for (int i = 0; i < width; i++)
        for (int j = 0; j < width; j++) {
            double ddx = fabs(j - center + delta), ddy = fabs(i - center + delta);
            double dis = sqrt(ddx * ddx + ddy * ddy);
            if (dis < radius + eps && dis > inner - eps) {
                r->in[i * width + j] = 1;
                r->dx[r->count] = j - center; r->dy[r->count] = i - center; r->count++;
            }
        }
    r->x1 = r->y1 = -center; r->x2 = r->y2 = width - center - 1;
}
/* SectorRange (Range.h:121-166) */
static void sector_range(Range *r, float angle, float radius, int parity) {
    const double PI = 3.1415926536, eps = 0.00001;
    int height = (int)(radius + 0.5);
    int width = (int)(2 * radius * sin(angle / 2 * (PI / 180)) + 0.5);
    if (width % 2 != parity) width--;
    r->w = width; r->h = height; range_alloc(r); r->count = 0;
    for (int i = 0; i < height; i++)
        for (int j = 0; j < width; j++) {
            double ddx = fabs(j - (width - 1) / 2.0), ddy = fabs((double)(height - i));
            double dis = sqrt(ddx * ddx + ddy * ddy);
            if (dis < radius + 0.2 + eps && ddx / ddy < tan(angle / 2 * PI / 180) + eps) {
                r->in[i * width + j] = 1;
                r->dx[r->count] = j - width / 2; r->dy[r->count] = i - height; r->count++;
            }
        }
    r->x1 = -width / 2; r->y1 = -height; r->x2 = (width - 1) / 2; r->y2 = -1;
}

/* ---------------------------------------------------------------- helpers ---- */
static int group2channel(const Env *e, int g) {       /* GridWorld.cc:999-1008 */
    return (e->food_mode ? 2 : 1) + g * (e->minimap_mode ? 3 : 2);
}
static int feature_size(const Env *e, int g) {        /* GridWorld.cc:1010-1018 */
    int f = e->embedding_size + e->types[e->groups[g].type].n_action + 1;
    if (e->goal_mode) f += 2;
    if (e->minimap_mode) f += 2;
    return f;
}
static Type *gtype(Env *e, int g) { return &e->types[e->groups[g].type]; }
static int cell_channel(const Env *e, int c) {         /* channel_ids view of the map */
    int v = e->cells[c];
    if (v == CELL_EMPTY) return -1;
    if (v == CELL_WALL) return 0;
    return group2channel(e, e->pool[v].group);
}
static bool blank(const Env *e, int x, int y, int self) {   /* Map.cc:466-482, 1x1 */
    if (x < 0 || y < 0 || x + 1 >= e->w || y + 1 >= e->h) return false;
    int v = e->cells[y * e->w + x];
    return v == CELL_EMPTY || v == self;
}

/* ---------------------------------------------------------------- C ABI ------ */
int env_new_game(void **game, const char *name) {
    if (strcmp(name, "GridWorld") != 0) ORC_FAIL("invalid name of game %s", name);
    Env *e = calloc(1, sizeof(Env));
    rng_seed(e, 0);                                    /* GridWorld.cc:31 */
    *game = e;
    return 0;
}

int env_delete_game(void *game) {
    Env *e = game;
    if (!e) return 0;
    for (int t = 0; t < e->n_types; t++) {
        Range *rs[3] = {&e->types[t].view, &e->types[t].attack, &e->types[t].move};
        for (int k = 0; k < 3; k++) { free(rs[k]->in); free(rs[k]->dx); free(rs[k]->dy); }
    }
    for (int g = 0; g < e->n_groups; g++) free(e->groups[g].ids);
    free(e->cells); free(e->pool); free(e->atk); free(e->mov);
    free(e);
    return 0;
}

int env_config_game(void *game, const char *key, void *p) {     /* GridWorld.cc:126-155 */
    Env *e = game;
    if (!strcmp(key, "map_width")) e->w = *(int *)p;
    else if (!strcmp(key, "map_height")) e->h = *(int *)p;
    else if (!strcmp(key, "food_mode")) e->food_mode = *(bool *)p;
    else if (!strcmp(key, "turn_mode")) e->turn_mode = *(bool *)p;
    else if (!strcmp(key, "minimap_mode")) e->minimap_mode = *(bool *)p;
    else if (!strcmp(key, "goal_mode")) e->goal_mode = *(bool *)p;
    else if (!strcmp(key, "embedding_size")) e->embedding_size = *(int *)p;
    else if (!strcmp(key, "render_dir")) { /* render is out of scope */ }
    else if (!strcmp(key, "seed")) rng_seed(e, (unsigned long)(long)*(int *)p);
    else ORC_FAIL("invalid argument in set_config: %s", key);
    if (e->food_mode || e->turn_mode || e->goal_mode) ORC_FAIL("food/turn/goal modes unsupported");
    return 0;
}

int gridworld_register_agent_type(void *game, const char *name, int n, const char **keys,
                                  float *values) {            /* AgentType.cc:28-131 */
    Env *e = game;
    if (e->n_types >= MAX_TYPES) ORC_FAIL("too many agent types");
    for (int t = 0; t < e->n_types; t++)
        if (!strcmp(e->types[t].name, name)) ORC_FAIL("duplicated agent type %s", name);
    Type *T = &e->types[e->n_types];
    memset(T, 0, sizeof(*T));
    snprintf(T->name, sizeof T->name, "%s", name);
    T->width = T->length = 1; T->speed = 1; T->hp = 1;
    T->view_radius = 1; T->view_angle = 360;
    for (int i = 0; i < n; i++) {
        const char *k = keys[i]; float v = values[i];
#define FI(f) if (!strcmp(k, #f)) { T->f = (int)(v + 0.5); continue; }
#define FF(f) if (!strcmp(k, #f)) { T->f = v; continue; }
#define FB(f) if (!strcmp(k, #f)) { T->f = (bool)(int)(v + 0.5); continue; }
        FI(width) FI(length) FF(speed) FF(hp) FF(view_radius) FF(view_angle)
        FF(attack_radius) FF(attack_angle) FF(hear_radius) FF(speak_radius) FI(speak_ability)
        FF(damage) FF(trace) FF(eat_ability) FF(step_recover) FF(kill_supply) FF(food_supply)
        FB(attack_in_group) FB(can_absorb) FF(step_reward) FF(kill_reward) FF(dead_penalty)
        FF(attack_penalty)
        if (!strcmp(k, "view_x_offset") || !strcmp(k, "view_y_offset") || !strcmp(k, "att_x_offset") ||
            !strcmp(k, "att_y_offset") || !strcmp(k, "turn_x_offset") || !strcmp(k, "turn_y_offset"))
            continue;   /* accepted, then overwritten below (AgentType.cc:117-120) */
#undef FI
#undef FF
#undef FB
        ORC_FAIL("invalid agent config %s", k);
    }
    if (T->width != 1 || T->length != 1) ORC_FAIL("only 1x1 agents supported");
    int parity = T->width % 2;
    if (T->view_angle >= 180) {
        if (fabs(T->view_angle - 360) > 1e-5) ORC_FAIL("angle must be 360 when > 180");
        circle_range(&T->view, T->view_radius, 0, parity);
    } else sector_range(&T->view, T->view_angle, T->view_radius, parity);
    if (T->attack_angle >= 180) {
        if (fabs(T->attack_angle - 360) > 1e-5) ORC_FAIL("angle must be 360 when > 180");
        circle_range(&T->attack, T->attack_radius, T->width / 2.0f, parity);
    } else sector_range(&T->attack, T->attack_angle, T->attack_radius, parity);
    circle_range(&T->move, T->speed, 0, 1);
    T->view_x_offset = T->width / 2; T->view_y_offset = T->length / 2;
    T->att_x_offset = T->width / 2; T->att_y_offset = T->length / 2;
    T->turn_base = T->move.count;
    T->attack_base = T->turn_base;
    T->n_action = T->attack_base + T->attack.count;
    e->n_types++;
    return 0;
}

int gridworld_new_group(void *game, const char *type_name, int *group) {
    Env *e = game;
    for (int t = 0; t < e->n_types; t++)
        if (!strcmp(e->types[t].name, type_name)) {
            if (e->n_groups >= MAX_GROUPS) ORC_FAIL("too many groups");
            Group *G = &e->groups[e->n_groups];
            memset(G, 0, sizeof *G);
            G->type = t;
            *group = e->n_groups++;
            return 0;
        }
    ORC_FAIL("invalid agent type %s", type_name);
}

int gridworld_define_agent_symbol(void *game, int no, int group, int index) {
    Env *e = game;
    if (no >= MAX_SYM) ORC_FAIL("too many symbols");
    e->syms[no].group = group; e->syms[no].index = index;
    if (no >= e->n_syms) e->n_syms = no + 1;
    return 0;
}

int gridworld_define_event_node(void *game, int no, int op, int *inputs, int n_inputs) {
    Env *e = game;
    if (no >= MAX_SYM || n_inputs > 8) ORC_FAIL("event node out of range");
    e->nodes[no].op = op; e->nodes[no].n_raw = n_inputs;
    for (int i = 0; i < n_inputs; i++) e->nodes[no].raw[i] = inputs[i];
    if (no >= e->n_nodes) e->n_nodes = no + 1;
    return 0;
}

/* The reference python passes 6 of the 7 arguments (gridworld.py:719-722): auto_value is
 * never read here (only OP_ALIGN uses it, RewardEngine.cc:252). */
int gridworld_add_reward_rule(void *game, int on, int *receivers, float *values, int n_receiver,
                              bool is_terminal, bool auto_value) {
    (void)auto_value;
    Env *e = game;
    if (e->n_rules >= MAX_RULES || n_receiver > 8) ORC_FAIL("too many rules/receivers");
    Rule *R = &e->rules[e->n_rules++];
    R->on = on; R->n_recv = n_receiver; R->terminal = is_terminal;
    for (int i = 0; i < n_receiver; i++) { R->recv[i] = receivers[i]; R->val[i] = values[i]; }
    return 0;
}

static int check_rules(Env *e) {
    for (int r = 0; r < e->n_rules; r++) {
        Rule *R = &e->rules[r];
        Node *N = &e->nodes[R->on];
        if (N->op != OP_ATTACK && N->op != OP_KILL && N->op != OP_COLLIDE)
            ORC_FAIL("reward rule %d: only attack/kill/collide events supported", r);
        Sym *a = &e->syms[N->raw[0]], *b = &e->syms[N->raw[1]];
        if (a->index != -1 || b->index != -1 || a->group == b->group)
            ORC_FAIL("reward rule %d: symbols must be 'any' of two different groups", r);
        for (int i = 0; i < R->n_recv; i++)
            if (R->recv[i] != N->raw[0] && R->recv[i] != N->raw[1])
                ORC_FAIL("reward rule %d: receiver must be the event subject or object", r);
    }
    return 0;
}

int env_reset(void *game) {                                   /* GridWorld.cc:76-124 */
    Env *e = game;
    if (e->w <= 0 || e->h <= 0) ORC_FAIL("map size not set");
    e->id_counter = 0;
    if (e->w * e->h > 99 * 99) {
        e->large_map_mode = true;
        e->n_sep = e->w * e->h > 1000 * 1000 ? 16 : 8;
    }
    free(e->cells);
    e->cells = malloc(sizeof(int) * (size_t)e->w * e->h);
    for (int i = 0; i < e->w * e->h; i++) e->cells[i] = CELL_EMPTY;
    for (int i = 0; i < e->w; i++) { e->cells[i] = CELL_WALL; e->cells[(e->h - 1) * e->w + i] = CELL_WALL; }
    for (int i = 0; i < e->h; i++) { e->cells[i * e->w] = CELL_WALL; e->cells[i * e->w + e->w - 1] = CELL_WALL; }
    e->n_pool = 0;
    for (int g = 0; g < e->n_groups; g++) { e->groups[g].n = 0; e->groups[g].dead_ct = 0; }
    e->n_atk = e->n_mov = 0;
    return check_rules(e);
}

static Agent *new_agent(Env *e, int g) {
    if (e->n_pool == e->cap_pool) {
        e->cap_pool = e->cap_pool ? 2 * e->cap_pool : 1024;
        e->pool = realloc(e->pool, sizeof(Agent) * (size_t)e->cap_pool);
    }
    Agent *a = &e->pool[e->n_pool];
    Type *T = gtype(e, g);
    memset(a, 0, sizeof *a);
    a->id = e->id_counter; a->group = g; a->hp = T->hp;
    a->last_action = T->n_action;                  /* GridWorld.h:145 */
    a->absorbed = false;                           /* GridWorld.h:136 */
    a->last_op = OP_NULL; a->op_obj = -1;
    a->last_reward = 0; a->next_reward = T->step_reward;   /* init_reward() in ctor */
    return a;
}

static void group_push(Group *G, int id) {
    if (G->n == G->cap) { G->cap = G->cap ? 2 * G->cap : 256; G->ids = realloc(G->ids, sizeof(int) * (size_t)G->cap); }
    G->ids[G->n++] = id;
}

static void add_one(Env *e, int g, int x, int y) {           /* Map.cc:75-97 + add_or_error */
    Agent *a = new_agent(e, g);
    if (!blank(e, x, y, -1)) return;                 /* silently ignored; id not consumed */
    a->x = x; a->y = y;
    e->cells[y * e->w + x] = a->id;
    e->n_pool++; e->id_counter++;
    group_push(&e->groups[g], a->id);
}

static int add_wall(Env *e, int x, int y) {                  /* Map.cc:108-115 */
    if (x < 0 || y < 0 || x >= e->w || y >= e->h) return 1;
    int *c = &e->cells[y * e->w + x];
    if (*c >= 0) return 1;
    *c = CELL_WALL;
    return 0;
}

static void random_blank(Env *e, int *x, int *y) {          /* Map.cc:49-63 (1x1) */
    for (int tries = 0;; tries++) {
        *x = (int)rng_next(e) % (e->w - 1);
        *y = (int)rng_next(e) % (e->h - 1);
        if (blank(e, *x, *y, -1)) return;
        if (tries > e->w * e->h) { fprintf(stderr, "battle_oracle: no blank position\n"); abort(); }
    }
}

int gridworld_add_agents(void *game, int group, int n, const char *method, const int *xs,
                         const int *ys, const int *dirs) {   /* GridWorld.cc:189-301 */
    (void)dirs;
    Env *e = game;
    if (!e->cells) ORC_FAIL("add_agents before reset");
    if (group == -1) {
        if (!strcmp(method, "random")) {
            for (int i = 0; i < n; i++) { int x, y; random_blank(e, &x, &y); add_wall(e, x, y); }
        } else if (!strcmp(method, "custom")) {
            for (int i = 0; i < n; i++) add_wall(e, xs[i], ys[i]);
        } else if (!strcmp(method, "fill")) {
            for (int x = xs[0]; x < xs[0] + xs[2]; x++)
                for (int y = xs[1]; y < xs[1] + xs[3]; y++) add_wall(e, x, y);
        } else ORC_FAIL("unsupported method %s", method);
        return 0;
    }
    if (group < 0 || group >= e->n_groups) ORC_FAIL("invalid group %d", group);
    if (!strcmp(method, "random")) {
        for (int i = 0; i < n; i++) { int x, y; random_blank(e, &x, &y); add_one(e, group, x, y); }
    } else if (!strcmp(method, "custom")) {
        for (int i = 0; i < n; i++) add_one(e, group, xs[i], ys[i]);
    } else if (!strcmp(method, "fill")) {
        for (int x = xs[0]; x < xs[0] + xs[2]; x++)
            for (int y = xs[1]; y < xs[1] + xs[3]; y++) add_one(e, group, x, y);
    } else ORC_FAIL("unsupported method %s", method);
    return 0;
}

/* get_observation: GridWorld.cc:303-426, Map.cc:130-218 (NORTH, 1x1) */
int env_get_observation(void *game, int group, float **bufs) {
    Env *e = game;
    Group *G = &e->groups[group];
    Type *T = gtype(e, group);
    const int n_group = e->n_groups, n_ch = group2channel(e, n_group);
    const int VW = T->view.w, VH = T->view.h, F = feature_size(e, group);
    const int n = G->n, n_action = T->n_action, emb = e->embedding_size;
    float *view = bufs[0], *feat = bufs[1];
    memset(view, 0, sizeof(float) * (size_t)n * VW * VH * n_ch);
    memset(feat, 0, sizeof(float) * (size_t)n * F);
    int trans[64];                                                     /* make_channel_trans */
    memset(trans, 0, sizeof trans);
    int base = group2channel(e, 0);
    for (int i = 0; i < base; i++) trans[i] = i;
    for (int i = 0; i < n_group; i++) {
        trans[group2channel(e, (group + i) % n_group)] = base;
        base += e->minimap_mode ? 3 : 2;
    }
    int scale_h = (e->h + VH - 1) / VH, scale_w = (e->w + VW - 1) / VW;
    float *mm = NULL;
    if (e->minimap_mode) {
        mm = calloc((size_t)VH * VW * n_group, sizeof(float));
        /* GridWorld.cc:357-363: absorbed agents are skipped when the OBSERVING group's type can absorb
           (the reference reads agents[0] of the observed group inside every group's loop) */
        const bool skip = T->can_absorb;
        for (int g = 0; g < n_group; g++) {
            Group *Gi = &e->groups[g];
            size_t total = 0;
            for (int j = 0; j < Gi->n; j++) {
                Agent *a = &e->pool[Gi->ids[j]];
                if (skip && a->absorbed) continue;
                mm[((a->y / scale_h) * VW + a->x / scale_w) * n_group + g] += 1.0f;
                total++;
            }
            for (int c = 0; c < VH * VW; c++) mm[c * n_group + g] /= (float)total;
        }
    }
    for (int i = 0; i < n; i++) {
        Agent *a = &e->pool[G->ids[i]];
        float *vb = view + (size_t)i * VW * VH * n_ch;
        int eye_x = a->x + T->view_x_offset, eye_y = a->y + T->view_y_offset;
        int x1 = eye_x + T->view.x1, y1 = eye_y + T->view.y1, x2 = eye_x + T->view.x2, y2 = eye_y + T->view.y2;
        int sx = x1 > 0 ? x1 : 0, ex = x2 < e->w - 1 ? x2 : e->w - 1;
        int sy = y1 > 0 ? y1 : 0, ey = y2 < e->h - 1 ? y2 : e->h - 1;
        for (int x = sx; x <= ex; x++)
            for (int y = sy; y <= ey; y++) {
                int vx = x - eye_x - T->view.x1, vy = y - eye_y - T->view.y1;
                int cid = cell_channel(e, y * e->w + x);
                if (cid != -1 && T->view.in[vy * VW + vx]) {
                    int ch = trans[cid];
                    vb[(vy * VW + vx) * n_ch + ch] = 1;
                    int v = e->cells[y * e->w + x];
                    if (v >= 0) {
                        Agent *o = &e->pool[v];
                        vb[(vy * VW + vx) * n_ch + ch + 1] = o->hp / gtype(e, o->group)->hp;
                    }
                }
            }
        if (e->minimap_mode) {
            int self_x = a->x / scale_w, self_y = a->y / scale_h;
            for (int j = 0; j < n_group; j++) {
                int mch = trans[group2channel(e, j)] + 2;
                for (int k = 0; k < VH; k++)
                    for (int l = 0; l < VW; l++) vb[(k * VW + l) * n_ch + mch] = mm[(k * VW + l) * n_group + j];
                vb[(self_y * VW + self_x) * n_ch + mch] += 1;
            }
        }
        float *fb = feat + (size_t)i * F;
        for (int k = 0, t = a->id; k < emb; k++, t >>= 1) fb[k] = (float)(t & 1);
        fb[emb + a->last_action] = 1;
        fb[emb + n_action] = a->last_reward;
        if (e->minimap_mode) {
            fb[emb + n_action + 1] = (float)a->x / e->w;
            fb[emb + n_action + 2] = (float)a->y / e->h;
        }
    }
    free(mm);
    return 0;
}

static void push_act(Act **buf, int *n, int *cap, Act a) {
    if (*n == *cap) { *cap = *cap ? 2 * *cap : 1024; *buf = realloc(*buf, sizeof(Act) * (size_t)*cap); }
    (*buf)[(*n)++] = a;
}

int env_set_action(void *game, int group, const int *actions) {   /* GridWorld.cc:430-496 */
    Env *e = game;
    Group *G = &e->groups[group];
    Type *T = gtype(e, group);
    int bw = e->large_map_mode ? (e->w + e->n_sep - 1) / e->n_sep : 1;
    for (int i = 0; i < G->n; i++) {
        Agent *a = &e->pool[G->ids[i]];
        int act = actions[i];
        if (act < 0 || act >= T->n_action) ORC_FAIL("invalid action %d", act);
        a->last_action = act;
        if (act < T->turn_base) {
            int bucket = -1;                      /* -1 = boundary buffer */
            if (e->large_map_mode) {
                int x_ = a->x % bw;
                if (!(x_ < 4 || x_ > bw - 4)) bucket = a->x / bw;
            }
            push_act(&e->mov, &e->n_mov, &e->cap_mov, (Act){a->id, act, bucket});
        } else {
            push_act(&e->atk, &e->n_atk, &e->cap_atk, (Act){a->id, act - T->attack_base, 0});
        }
    }
    return 0;
}

static void do_move(Env *e, Act *m) {                          /* GridWorld.cc:631-660, Map.cc:324-369 */
    Agent *a = &e->pool[m->id];
    if (a->dead || a->absorbed) return;                         /* GridWorld.cc:638 */
    Type *T = gtype(e, a->group);
    int nx = a->x + T->move.dx[m->action], ny = a->y + T->move.dy[m->action];
    if (blank(e, nx, ny, a->id)) {
        e->cells[a->y * e->w + a->x] = CELL_EMPTY;
        e->cells[ny * e->w + nx] = a->id;
        a->x = nx; a->y = ny;
    } else if (nx >= 0 && ny >= 0 && nx + 1 < e->w && ny + 1 < e->h) {
        int v = e->cells[ny * e->w + nx];
        if (v >= 0 && v != a->id) {
            Agent *o = &e->pool[v];
            if (gtype(e, o->group)->can_absorb) {                   /* Map.cc:352-359 */
                if (!o->absorbed) {
                    o->absorbed = true;
                    o->hp = o->hp * 2;
                    a->dead = true;
                    e->cells[a->y * e->w + a->x] = CELL_EMPTY;          /* Map::remove_agent */
                    a->last_op = OP_COLLIDE; a->op_obj = v;
                }
            } else {
                a->last_op = OP_COLLIDE; a->op_obj = v;
            }
        }
    }
}

int env_step(void *game, int *done) {                          /* GridWorld.cc:498-694 */
    Env *e = game;
    /* shuffle attacks (:507-515) */
    for (int i = 0; i < e->n_atk; i++) {
        int j = (int)rng_next(e) % (i + 1);
        Act t = e->atk[i]; e->atk[i] = e->atk[j]; e->atk[j] = t;
    }
    /* attack (:521-558), sequential */
    for (int i = 0; i < e->n_atk; i++) {
        Agent *a = &e->pool[e->atk[i].id];
        if (a->dead) continue;
        Type *T = gtype(e, a->group);
        int ox = a->x + T->att_x_offset + T->attack.dx[e->atk[i].action];
        int oy = a->y + T->att_y_offset + T->attack.dy[e->atk[i].action];
        int v = (ox >= 0 && ox < e->w && oy >= 0 && oy < e->h) ? e->cells[oy * e->w + ox] : CELL_EMPTY;
        if (v < 0 || (!T->attack_in_group && e->pool[v].group == a->group)) {
            a->next_reward += T->attack_penalty;                /* blank */
            continue;
        }
        Agent *o = &e->pool[v];
        Type *OT = gtype(e, o->group);
        float reward = 0.0f;
        o->hp -= T->damage;                                     /* be_attack GridWorld.h:208-214 */
        if (o->hp < 0.0) {
            o->dead = true;
            o->next_reward = OT->dead_penalty;
            a->last_op = OP_KILL; a->op_obj = o->id;
            e->cells[o->y * e->w + o->x] = CELL_EMPTY;
            e->groups[o->group].dead_ct++;
            float hp2 = a->hp + OT->kill_supply;                /* add_hp GridWorld.h:190 */
            a->hp = T->hp < hp2 ? T->hp : hp2;
            reward = OT->kill_reward;
        } else {
            a->last_op = OP_ATTACK; a->op_obj = o->id;
        }
        a->next_reward += reward + T->attack_penalty;
    }
    e->n_atk = 0;
    /* starve (:570-595) */
    for (int g = 0; g < e->n_groups; g++) {
        Group *G = &e->groups[g];
        Type *T = gtype(e, g);
        for (int j = 0; j < G->n; j++) {
            Agent *a = &e->pool[G->ids[j]];
            if (a->dead) continue;
            if (T->step_recover > 0) {
                float hp2 = a->hp + T->step_recover;
                a->hp = T->hp < hp2 ? T->hp : hp2;
            } else {
                a->hp -= -T->step_recover;
                if (a->hp < 0.0) { a->dead = true; a->next_reward = T->dead_penalty; }
            }
            if (a->dead) { e->cells[a->y * e->w + a->x] = CELL_EMPTY; G->dead_ct++; }
        }
    }
    /* move (:628-672): large map: band buffers 0..n_sep-1 then the boundary buffer */
    if (e->large_map_mode)
        for (int b = 0; b < e->n_sep; b++)
            for (int i = 0; i < e->n_mov; i++) if (e->mov[i].bucket == b) do_move(e, &e->mov[i]);
    for (int i = 0; i < e->n_mov; i++) if (e->mov[i].bucket == -1) do_move(e, &e->mov[i]);
    e->n_mov = 0;
    /* calc_reward (:744-758, RewardEngine.cc:373-443): supported subset */
    for (int r = 0; r < e->n_rules; r++) {
        Rule *R = &e->rules[r];
        Node *N = &e->nodes[R->on];
        int sa = N->raw[0], sb = N->raw[1];
        Group *G = &e->groups[e->syms[sa].group];
        e->rule_trigger[r] = false;
        for (int j = 0; j < G->n; j++) {
            Agent *a = &e->pool[G->ids[j]];
            if (a->op_obj < 0 || e->pool[a->op_obj].group != e->syms[sb].group) continue;
            if (a->last_op != N->op) continue;
            e->rule_trigger[r] = true;
            for (int k = 0; k < R->n_recv; k++) {
                Agent *rcv = R->recv[k] == sa ? a : &e->pool[a->op_obj];
                rcv->next_reward += R->val[k];
            }
        }
    }
    int live = 0;
    for (int g = 0; g < e->n_groups; g++) if (e->groups[g].n - e->groups[g].dead_ct > 0) live++;
    *done = live < e->n_groups;
    for (int r = 0; r < e->n_rules; r++) if (e->rule_trigger[r] && e->rules[r].terminal) *done = 1;
    return 0;
}

int gridworld_clear_dead(void *game) {                        /* GridWorld.cc:696-728 */
    Env *e = game;
    for (int g = 0; g < e->n_groups; g++) {
        Group *G = &e->groups[g];
        G->reward = 0;
        int pt = 0;
        for (int j = 0; j < G->n; j++) {
            Agent *a = &e->pool[G->ids[j]];
            if (a->dead) continue;
            a->last_reward = a->next_reward;                      /* init_reward GridWorld.h:173-179 */
            a->last_op = OP_NULL; a->op_obj = -1;
            a->next_reward = gtype(e, g)->step_reward;
            a->index = pt;
            G->ids[pt++] = a->id;
        }
        G->n = pt;
        G->dead_ct = 0;
    }
    return 0;
}

int env_get_reward(void *game, int group, float *buf) {       /* GridWorld.cc:760-770 */
    Env *e = game;
    Group *G = &e->groups[group];
    for (int i = 0; i < G->n; i++) buf[i] = e->pool[G->ids[i]].next_reward + G->reward;
    return 0;
}

int env_get_info(void *game, int group, const char *name, void *buffer) {   /* GridWorld.cc:777-978 */
    Env *e = game;
    int *ib = buffer; bool *bb = buffer;
    if (!strcmp(name, "num")) { ib[0] = e->groups[group].n; return 0; }
    if (!strcmp(name, "id")) { for (int i = 0; i < e->groups[group].n; i++) ib[i] = e->groups[group].ids[i]; return 0; }
    if (!strcmp(name, "pos")) {
        for (int i = 0; i < e->groups[group].n; i++) {
            Agent *a = &e->pool[e->groups[group].ids[i]];
            ib[2 * i] = a->x; ib[2 * i + 1] = a->y;
        }
        return 0;
    }
    if (!strcmp(name, "alive")) {
        for (int i = 0; i < e->groups[group].n; i++) bb[i] = !e->pool[e->groups[group].ids[i]].dead;
        return 0;
    }
    /* not a reference key: the hp of every group member (the rollout replays compare the state with it) */
    if (!strcmp(name, "hp")) {
        float *fb = buffer;
        for (int i = 0; i < e->groups[group].n; i++) fb[i] = e->pool[e->groups[group].ids[i]].hp;
        return 0;
    }
    if (!strcmp(name, "action_space")) { ib[0] = gtype(e, group)->n_action; return 0; }
    if (!strcmp(name, "view_space")) {
        ib[0] = gtype(e, group)->view.h; ib[1] = gtype(e, group)->view.w; ib[2] = group2channel(e, e->n_groups);
        return 0;
    }
    if (!strcmp(name, "feature_space")) { ib[0] = feature_size(e, group); return 0; }
    if (!strcmp(name, "attack_base")) { ib[0] = gtype(e, group)->attack_base; return 0; }
    if (!strcmp(name, "view2attack")) {
        Type *T = gtype(e, group);
        for (int i = 0; i < T->view.w * T->view.h; i++) ib[i] = -1;
        for (int i = 0; i < T->attack.count; i++)
            ib[(T->attack.dy[i] - T->view.y1) * T->view.w + (T->attack.dx[i] - T->view.x1)] = i;
        return 0;
    }
    if (!strcmp(name, "both_attack")) { ib[0] = 0; return 0; }
    ORC_FAIL("unsupported info name %s", name);
}

int env_render(void *game) { (void)game; return 0; }
int env_render_next_file(void *game) { (void)game; return 0; }
int gridworld_set_goal(void *game, int group, const char *method, const int *buf) {
    (void)game; (void)group; (void)method; (void)buf;
    ORC_FAIL("set_goal is deprecated/unsupported");
}
