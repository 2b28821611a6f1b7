// scene.cpp — the product scene compiler: reference scene JSON -> rmr tables.
//
// The reference generates GLSL source per scene and lets the GL driver reject it:
//   v1 objects   Graphics.cpp:647-702  (obj_func_<j>, //#OBJFUNCINSERT, //#OBJINSERT 94-113)
//   v1 materials Graphics.cpp:513-645  (mat_func_<id>, //#CASEINSERT 69-88)
//   v2 materials Graphics.cpp:392-509 + 705-739 (mat_func_<id> for RayMarch2.glsl)
// Here the same node lists become table rows that the kernels interpret; every condition under
// which the generated GLSL would not compile is reported as a SceneError instead.
#include "scene.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>

namespace rmr {

namespace {

// std::to_string(input.asFloat()) == "%f", then parsed back as a GLSL float literal
float quant_v1(double x) {
    char buf[64];
    std::snprintf(buf, sizeof buf, "%f", (double)(float)x);
    return (float)std::strtod(buf, nullptr);
}

struct NodeSig { int code, n_in, n_out; };

const std::map<std::string, NodeSig>& obj_nodes() {  // RayMarch.glsl:121-215
    static const std::map<std::string, NodeSig> m = {
        {"misc_getX", {RMR_OP_GET_X, 1, 1}}, {"misc_getY", {RMR_OP_GET_Y, 1, 1}}, {"misc_getZ", {RMR_OP_GET_Z, 1, 1}},
        {"math_add", {RMR_OP_ADD, 2, 1}}, {"math_subtract", {RMR_OP_SUB, 2, 1}},
        {"math_multiply", {RMR_OP_MUL, 2, 1}}, {"math_divide", {RMR_OP_DIV, 2, 1}},
        {"math_sine", {RMR_OP_SIN, 1, 1}}, {"math_cosine", {RMR_OP_COS, 1, 1}},
        {"map_sphere", {RMR_OP_MAP_SPHERE, 3, 1}}, {"map_box", {RMR_OP_MAP_BOX, 3, 1}},
        {"op_union", {RMR_OP_UNION, 2, 1}}, {"op_subtract", {RMR_OP_SUBTRACT, 2, 1}},
        {"op_intersect", {RMR_OP_INTERSECT, 2, 1}}, {"domain_repeat", {RMR_OP_DOMAIN_REPEAT, 2, 1}},
        {"map_mandelbulb", {RMR_OP_MAP_MANDELBULB, 3, 1}},  // rmr extension
    };
    return m;
}
const std::map<std::string, NodeSig>& mat_nodes() {  // RayMarch.glsl:313-479
    static const std::map<std::string, NodeSig> m = {
        {"misc_facing", {RMR_OP_M_FACING, 0, 1}}, {"misc_inside", {RMR_OP_M_INSIDE, 0, 1}},
        {"math_add", {RMR_OP_M_ADD, 2, 1}}, {"math_subtract", {RMR_OP_M_SUB, 2, 1}},
        {"math_multiply", {RMR_OP_M_MUL, 2, 1}}, {"math_divide", {RMR_OP_M_DIV, 2, 1}},
        {"shader_mix", {RMR_OP_M_MIX, 7, 3}}, {"shader_diffuse", {RMR_OP_M_DIFFUSE, 1, 2}},
        {"shader_glossy", {RMR_OP_M_GLOSSY, 2, 2}}, {"shader_refraction", {RMR_OP_M_REFRACTION, 3, 3}},
        {"shader_volumeScatter", {RMR_OP_M_VOLUME, 2, 4}}, {"shader_emission", {RMR_OP_M_EMISSION, 2, 1}},
    };
    return m;
}

int prim_fast_type(const std::string& n) {
    if (n == "map_sphere") return RMR_PRIM_SPHERE;
    if (n == "map_box") return RMR_PRIM_BOX;
    if (n == "map_mandelbulb") return RMR_PRIM_MANDELBULB;
    return 0;
}

rmr_op make_op(int code) {
    rmr_op o;
    o.code = code;
    for (int i = 0; i < 7; i++) o.in[i] = RMR_OPND_NONE;
    for (int i = 0; i < 4; i++) o.out[i] = -1;
    return o;
}

struct Builder {
    CompiledScene& sc;
    int add_const(float x, float y, float z) {
        sc.consts.push_back(x);
        sc.consts.push_back(y);
        sc.consts.push_back(z);
        return RMR_OPND_CONST0 - (int)(sc.consts.size() / 3 - 1);
    }
};

void literal3(const json::Value& a, float out[3]) {  // "vec3(%f, %f, %f)" of a JSON array
    for (int i = 0; i < 3; i++) out[i] = quant_v1(a[i].as_double());
}

int total_vars(const json::Value& o, const std::string& what) {
    const json::Value& tv = o.get("total_vars");
    if (!tv.is_int() || tv.i <= 0) throw SceneError(what + ": total_vars must be a positive int (vec3 vars[total_vars])");
    if (tv.i > RMR_MAX_VARS) throw SceneError(what + ": total_vars exceeds RMR_MAX_VARS");
    return (int)tv.i;
}
int check_var(long long k, int tv, const std::string& what) {
    if (k < 0 || k >= tv)
        throw SceneError(what + ": vars[" + std::to_string(k) + "] out of range for vec3 vars[" + std::to_string(tv) + "]");
    return (int)k;
}

struct Arg { char kind; int var; float lit[3]; };  // kind: 'c' literal, 'p' = p, 'v' var

void compile_objects_v1(CompiledScene& sc, const json::Value& objects) {
    Builder b{sc};
    for (size_t j = 0; j < objects.size(); j++) {
        const json::Value& obj = objects[j];
        const std::string what = "object " + std::to_string(j);
        const int tv = total_vars(obj, what);
        const json::Value& nodes = obj.get("nodes");
        const json::Value& dist = obj.get("distance");
        if (!dist.is_int()) throw SceneError(what + ": distance must be an int var index");
        check_var(dist.i, tv, what);
        const json::Value& mv = obj.get("matID");
        const float mat = mv.is_int() ? (float)mv.i : 0.0f;
        if (nodes.size() == 1 && prim_fast_type(nodes[0].get("name").s) != 0 && nodes[0].get("name").is_string()) {
            const json::Value& n = nodes[0];
            const json::Value& ins = n.get("inputs");
            const json::Value& outs = n.get("outputs");
            if (ins.size() == 3 && ins[0].is_int() && ins[0].i == -1 && ins[1].is_array() && ins[2].is_array() &&
                outs.size() == 1 && outs[0].is_int() && outs[0].i == dist.i) {
                rmr_prim p{};
                p.type = prim_fast_type(n.get("name").s);
                p.mat_id = mat;
                literal3(ins[1], p.c);
                literal3(ins[2], p.r);
                p.dist_var = (int)dist.i;
                p.n_vars = tv;
                sc.prims.push_back(p);
                continue;
            }
        }
        const int begin = (int)sc.ops.size();
        for (size_t k = 0; k < nodes.size(); k++) {
            const json::Value& n = nodes[k];
            const std::string name = n.get("name").is_string() ? n.get("name").s : std::string("?");
            auto it = obj_nodes().find(name);
            if (it == obj_nodes().end()) throw SceneError(what + ": no GLSL function '" + name + "'");
            const NodeSig sig = it->second;
            std::vector<Arg> args;
            const json::Value& ins = n.get("inputs");
            for (size_t a = 0; a < ins.size(); a++) {
                const json::Value& x = ins[a];
                Arg g{};
                if (x.is_array()) { g.kind = 'c'; literal3(x, g.lit); }
                else if (x.is_int()) {
                    if (x.i == -1) g.kind = 'p';
                    else { g.kind = 'v'; g.var = check_var(x.i, tv, what); }
                } else throw SceneError(what + ": object input is not an int or literal");
                args.push_back(g);
            }
            const json::Value& outs = n.get("outputs");
            for (size_t a = 0; a < outs.size(); a++) {
                if (!outs[a].is_int()) throw SceneError(what + ": object output is not an int");
                Arg g{};
                g.kind = 'v';
                g.var = check_var(outs[a].i, tv, what);
                args.push_back(g);
            }
            if ((int)args.size() != sig.n_in + sig.n_out)
                throw SceneError(what + ": " + name + " takes " + std::to_string(sig.n_in + sig.n_out) +
                                 " arguments, got " + std::to_string(args.size()));
            rmr_op op = make_op(sig.code);
            for (int i = 0; i < (int)args.size(); i++) {
                const Arg& g = args[i];
                if (i < sig.n_in) {
                    op.in[i] = g.kind == 'c' ? b.add_const(g.lit[0], g.lit[1], g.lit[2])
                                             : (g.kind == 'p' ? RMR_OPND_P : g.var);
                } else {
                    if (g.kind != 'v') throw SceneError(what + ": " + name + " out argument is not an l-value");
                    op.out[i - sig.n_in] = g.var;
                }
            }
            sc.ops.push_back(op);
        }
        rmr_prim p{};
        p.type = RMR_PRIM_PROGRAM;
        p.mat_id = mat;
        p.prog_begin = begin;
        p.prog_end = (int)sc.ops.size();
        p.dist_var = (int)dist.i;
        p.n_vars = tv;
        sc.prims.push_back(p);
    }
}

void compile_materials_v1(CompiledScene& sc, const json::Value& materials) {
    Builder b{sc};
    const size_t n = materials.size();
    std::map<long long, size_t> by_id;
    for (size_t i = 0; i < n; i++) {
        const json::Value& id = materials[i].get("id");
        if (!id.is_int()) throw SceneError("material id is not an int");
        if (by_id.count(id.i)) throw SceneError("mat_func_" + std::to_string(id.i) + " redefined");
        by_id[id.i] = i;
    }
    for (size_t j = 0; j < n; j++)
        if (!by_id.count((long long)j)) throw SceneError("case " + std::to_string(j) + " calls undefined mat_func_" + std::to_string(j));
    std::vector<rmr_material> out(n);
    for (size_t mi = 0; mi < n; mi++) {  // generation order = file order
        const json::Value& m = materials[mi];
        const long long mid = m.get("id").i;
        const std::string what = "material " + std::to_string(mid);
        const int tv = total_vars(m, what);
        std::map<std::string, int> names;
        const int begin = (int)sc.ops.size();
        const json::Value& nodes = m.get("nodes");
        for (size_t k = 0; k < nodes.size(); k++) {
            const json::Value& nd = nodes[k];
            const std::string name = nd.get("name").is_string() ? nd.get("name").s : std::string("?");
            auto it = mat_nodes().find(name);
            if (it == mat_nodes().end()) throw SceneError(what + ": no GLSL function " + name + "(RayData, ...)");
            const NodeSig sig = it->second;
            std::vector<Arg> args;
            const json::Value& ins = nd.get("inputs");
            for (size_t a = 0; a < ins.size(); a++) {
                const json::Value& x = ins[a];
                Arg g{};
                if (x.is_array()) { g.kind = 'c'; literal3(x, g.lit); args.push_back(g); }
                else if (x.is_string()) {
                    auto f = names.find(x.s);
                    if (f != names.end()) { g.kind = 'v'; g.var = f->second; args.push_back(g); }
                    // unknown names are dropped by the generator (Graphics.cpp:546-550)
                } else if (x.is_int()) { g.kind = 'v'; g.var = (int)x.i; args.push_back(g); }
            }
            const json::Value& outs = nd.get("outputs");
            for (size_t a = 0; a < outs.size(); a++) {
                const json::Value& x = outs[a];
                Arg g{};
                if (x.is_string()) {
                    auto f = names.find(x.s);
                    if (f == names.end()) { int idx = (int)names.size(); names[x.s] = idx; g.var = idx; }
                    else g.var = f->second;
                    g.kind = 'v';
                    args.push_back(g);
                } else if (x.is_int()) { g.kind = 'v'; g.var = (int)x.i; args.push_back(g); }
            }
            if ((int)args.size() != sig.n_in + sig.n_out)
                throw SceneError(what + ": " + name + " takes " + std::to_string(sig.n_in + sig.n_out) +
                                 " arguments, got " + std::to_string(args.size()));
            rmr_op op = make_op(sig.code);
            for (int i = 0; i < (int)args.size(); i++) {
                const Arg& g = args[i];
                if (g.kind == 'v') check_var(g.var, tv, what);
                if (i < sig.n_in) {
                    op.in[i] = g.kind == 'c' ? b.add_const(g.lit[0], g.lit[1], g.lit[2]) : g.var;
                } else {
                    if (g.kind != 'v') throw SceneError(what + ": " + name + " out argument is not an l-value");
                    op.out[i - sig.n_in] = g.var;
                }
            }
            sc.ops.push_back(op);
        }
        auto slot = [&](const char* key) -> int {
            const json::Value& v = m.get(key);
            if (v.is_string()) {
                auto f = names.find(v.s);
                int k = (f == names.end()) ? 0 : f->second;  // std::map::operator[] default (Graphics.cpp:592)
                return check_var(k, tv, what);
            }
            if (v.is_int() && v.i != -1) return check_var(v.i, tv, what);
            return -1;
        };
        rmr_material mm{};
        mm.defined = 1;
        mm.prog_begin = begin;
        mm.prog_end = (int)sc.ops.size();
        mm.n_vars = tv;
        mm.color_var = slot("color");
        mm.dir_var = slot("dir");
        mm.inside_var = slot("inside");
        mm.hit_var = slot("hit");
        out[(size_t)mid] = mm;
    }
    sc.materials = out;
}

// v2 slots: 0 newDir, 1 reflectance, 2/3 mixDir[0]/mixRefl[0], 4/5 mixDir[1]/mixRefl[1], 6 mixFact
struct V2Compiler {
    CompiledScene& sc;
    const json::Value& m;
    std::string what;
    int const_ref(const json::Value& inp, int want /*0 any, 1 vec3, 2 scalar*/) {
        if (!(inp.is_array() && inp.size() == 2 && inp[0].is_int() && inp[0].i == -1))
            throw SceneError(what + ": getInput() has no value for a node-linked input (Graphics.cpp:406)");
        const json::Value& consts = m.get("constants");
        const json::Value& k = inp[1];
        if (!k.is_int() || k.i < 0 || (size_t)k.i >= consts.size()) throw SceneError(what + ": constant missing");
        const json::Value& c = consts[(size_t)k.i];
        Builder b{sc};
        if (c.is_array()) {
            if (want == 2) throw SceneError(what + ": vec3 constant where a float is required");
            return b.add_const((float)c[0].as_double(), (float)c[1].as_double(), (float)c[2].as_double());
        }
        if (want == 1) throw SceneError(what + ": float constant where a vec3 is required");
        float f = (float)c.as_double();
        return b.add_const(f, f, f);
    }
    void node(const json::Value& idx, int out0, int out1, int depth, bool vec_kind) {
        const json::Value& nodes = m.get("nodes");
        if (!idx.is_int() || idx.i < 0 || (size_t)idx.i >= nodes.size()) throw SceneError(what + ": node missing");
        const json::Value& nd = nodes[(size_t)idx.i];
        const std::string name = nd.get("name").is_string() ? nd.get("name").s : std::string();
        const json::Value& ins = nd.get("inputs");
        if (name == "shader_diffuse") {
            if (!vec_kind) throw SceneError(what + ": shader_diffuse feeds a float");
            rmr_op o = make_op(RMR_OP_V2_DIFFUSE);
            o.in[0] = const_ref(ins[0], 1);
            o.out[0] = out0; o.out[1] = out1;
            sc.ops.push_back(o);
        } else if (name == "shader_glossy") {
            if (!vec_kind) throw SceneError(what + ": shader_glossy feeds a float");
            rmr_op o = make_op(RMR_OP_V2_GLOSSY);
            o.in[0] = const_ref(ins[0], 0);
            o.in[1] = const_ref(ins[1], 2);
            o.out[0] = out0; o.out[1] = out1;
            sc.ops.push_back(o);
        } else if (name == "shader_mix") {
            if (depth > 0 || !vec_kind) throw SceneError(what + ": nested shader_mix does not compile (Graphics.cpp:428-430)");
            const int o0s[3] = {2, 4, 6}, o1s[3] = {3, 5, -1};
            for (int i = 0; i < 3; i++) {
                const json::Value& inp = ins[(size_t)i];
                if (inp.is_array() && inp.size() >= 1 && inp[0].is_int() && inp[0].i != -1)
                    node(inp[0], o0s[i], o1s[i], depth + 1, i < 2);
            }
            rmr_op o = make_op(RMR_OP_V2_MIX);
            o.in[0] = 2; o.in[1] = 3; o.in[2] = 4; o.in[3] = 5; o.in[4] = 6;
            o.out[0] = out0; o.out[1] = out1;
            sc.ops.push_back(o);
        } else if (name == "misc_fresnel") {
            if (vec_kind) throw SceneError(what + ": misc_fresnel output assigned to a vec3");
            rmr_op o = make_op(RMR_OP_V2_FRESNEL);
            o.out[0] = out0;
            sc.ops.push_back(o);
        }
        // any other node name: compileNode emits nothing (Graphics.cpp:412-463)
    }
};

void builtin_prim(CompiledScene& sc, int type, float cx, float cy, float cz, float rx, float ry, float rz, int mat) {
    rmr_prim p{};
    p.type = type;
    p.mat_id = (float)mat;
    p.c[0] = cx; p.c[1] = cy; p.c[2] = cz;
    p.r[0] = rx; p.r[1] = ry; p.r[2] = rz;
    p.dist_var = 0;
    p.n_vars = 1;
    sc.prims.push_back(p);
}

void rm2_builtin(CompiledScene& sc) {
    builtin_prim(sc, RMR_PRIM_SPHERE, 0, 1, 0, 1, 1, 1, 1);  // RayMarch2.glsl:139
    std::memset(&sc.rm2, 0, sizeof sc.rm2);
    const float alb[3][3] = {{0.8f, 0.8f, 0.8f}, {0.8f, 0.2f, 0.2f}, {0.2f, 0.2f, 0.8f}};  // RayMarch2.glsl:445-456
    for (int i = 0; i < 3; i++)
        for (int c = 0; c < 3; c++) sc.rm2.albedo[i][c] = alb[i][c];
    sc.rm2.light_pos[0] = 2.0f; sc.rm2.light_pos[1] = 6.0f; sc.rm2.light_pos[2] = -2.0f;  // RayMarch2.glsl:458
    sc.rm2.light_power = 50.0f;                                                           // RayMarch2.glsl:459
    sc.rm2.node_mat_id = 1;                                                               // RayMarch2.glsl:463
}

void rm3_builtin(CompiledScene& sc) {
    builtin_prim(sc, RMR_PRIM_BOX, 0, -0.025f, 0, 32, 0.05f, 32, 1);  // RayMarch3.glsl:136
    builtin_prim(sc, RMR_PRIM_SPHERE, 0, 1, 0, 1, 1, 1, 2);           // RayMarch3.glsl:138
    builtin_prim(sc, RMR_PRIM_SPHERE, 6, 8, -4, 4, 4, 4, 0);          // RayMarch3.glsl:140
    auto spec = [](uint32_t mn, uint32_t mx, float p, int term) {
        rmr_spectral s{};
        s.defined = 1; s.min_wave = mn; s.max_wave = mx; s.power = p; s.terminates = term;
        return s;
    };
    sc.spectral = {spec(380, 780, 8.0f, 1),    // mat_func_0, RayMarch3.glsl:251-281
                   spec(380, 780, 0.8f, 0),    // mat_func_1, 283-313
                   spec(490, 590, 0.8f, 0)};   // mat_func_2, 315-345
    sc.spectral_sky = spec(390, 830, 0.015f, 0);  // RayMarch3.glsl:408-438
}

}  // namespace

rmr_scene CompiledScene::view() const {
    rmr_scene s{};
    s.variant = variant;
    s.n_prims = (int32_t)prims.size();
    s.prims = prims.data();
    s.n_ops = (int32_t)ops.size();
    s.ops = ops.data();
    s.n_consts = (int32_t)(consts.size() / 3);
    s.consts = consts.data();
    s.n_materials = (int32_t)(variant == RMR_VARIANT_RM3 ? spectral.size() : materials.size());
    s.materials = materials.data();
    s.spectral = spectral.data();
    s.spectral_sky = spectral_sky;
    s.v2_prog_begin = v2_begin;
    s.v2_prog_end = v2_end;
    s.v2_n_slots = v2_slots;
    s.rm2 = &rm2;
    for (int i = 0; i < 3; i++) s.sky[i] = sky[i];
    return s;
}

void CompiledScene::from_tables(const rmr_scene& s) {
    variant = s.variant;
    prims.assign(s.prims, s.prims + s.n_prims);
    ops.assign(s.ops, s.ops + s.n_ops);
    consts.assign(s.consts, s.consts + 3 * s.n_consts);
    materials.clear();
    spectral.clear();
    if (s.variant == RMR_VARIANT_RM3) {
        if (s.spectral) spectral.assign(s.spectral, s.spectral + s.n_materials);
    } else if (s.materials) {
        materials.assign(s.materials, s.materials + s.n_materials);
    }
    spectral_sky = s.spectral_sky;
    v2_begin = s.v2_prog_begin;
    v2_end = s.v2_prog_end;
    v2_slots = s.v2_n_slots;
    if (s.rm2) rm2 = *s.rm2; else std::memset(&rm2, 0, sizeof rm2);
    for (int i = 0; i < 3; i++) sky[i] = s.sky[i];
}

float max_sphere_radius(const CompiledScene& s) {
    float r = 0.0f;
    for (const rmr_prim& q : s.prims)
        if (q.type == RMR_PRIM_SPHERE) r = std::max(r, std::fabs(q.r[0]));
    return r;
}

// Algorithmic flops of one map() (add/sub/mul/min/max/abs/compare 1, FMA 2, sqrt 1 (+1
// transcendental), division 1): sphere 10, box 22, opU fold 2 per primitive after the first, a node
// program ~10 per node. A Mandelbulb primitive's fixed part is 6 (p - c; 0.5 log(r) r / dr); its
// iterations — 27 flops and 10 transcendentals each (length 6, bailout test 1, z.z / r 1, log-guard
// tests 2, power - 1 1, two exponent products 2, dr fma 3, angle scaling 2, direction products 2,
// z = dir zr + p0 6; sqrt, acos, atan2, log, exp x2, sin x2, cos x2) — depend on the point and are
// counted at run time by the RMR_COUNT_FLOPS build (rmr_trace.h).
double CompiledScene::flops_per_map() const {
    double f = 0;
    for (const auto& p : prims) {
        if (p.type == RMR_PRIM_SPHERE) f += 10;
        else if (p.type == RMR_PRIM_BOX) f += 22;
        else if (p.type == RMR_PRIM_MANDELBULB) f += 6;
        else f += 10.0 * std::max(1, p.prog_end - p.prog_begin);
    }
    return f + 2.0 * std::max<double>(0, (double)prims.size() - 1);
}
double CompiledScene::transc_per_map() const {
    double t = 0;
    for (const auto& p : prims) t += (p.type == RMR_PRIM_PROGRAM) ? 0.0 : 1.0;
    return t;
}

CompiledScene compile_scene(const std::string& text, int variant) {
    json::Value root;
    try {
        root = json::parse(text);
    } catch (const std::exception& e) {
        throw SceneError(e.what());
    }
    CompiledScene sc;
    sc.variant = variant;
    if (variant == RMR_VARIANT_RM1) {
        compile_objects_v1(sc, root.get("objects"));
        compile_materials_v1(sc, root.get("materials"));
    } else if (variant == RMR_VARIANT_RM2) {
        rm2_builtin(sc);
        bool found = false;
        const json::Value& mats = root.get("materials");
        for (size_t i = 0; i < mats.size(); i++) {
            const json::Value& m = mats[i];
            V2Compiler c{sc, m, "v2 material " + std::to_string(m.get("id").i)};
            const int begin = (int)sc.ops.size();
            c.node(m.get("output"), 0, 1, 0, true);
            if (m.get("id").is_int() && m.get("id").i == 1) {
                sc.v2_begin = begin;
                sc.v2_end = (int)sc.ops.size();
                found = true;
            }
        }
        if (!found) throw SceneError("RayMarch2.glsl calls mat_func_1, which the scene does not define");
        sc.v2_slots = 7;
    } else if (variant == RMR_VARIANT_RM3) {
        rm3_builtin(sc);  // RayMarch3.glsl has no insertion markers: generated text is discarded
    } else {
        throw SceneError("unknown variant " + std::to_string(variant));
    }
    if (sc.prims.size() > RMR_MAX_PRIMS || sc.ops.size() > RMR_MAX_OPS || sc.consts.size() / 3 > RMR_MAX_CONSTS)
        throw SceneError("scene exceeds table limits");
    return sc;
}

CompiledScene builtin_scene(int variant) {
    CompiledScene sc;
    sc.variant = variant;
    if (variant == RMR_VARIANT_RM3) rm3_builtin(sc);
    else if (variant == RMR_VARIANT_RM2) rm2_builtin(sc);
    else throw SceneError("RayMarch.glsl has no built-in scene (its map() is generated)");
    return sc;
}

}  // namespace rmr

// ---- context-free C ABI ----------------------------------------------------------------------
struct rmr_scene_blob {
    rmr::CompiledScene sc;
};

extern "C" int rmr_scene_compile(int variant, const char* json, size_t len, rmr_scene_blob** out, char* err,
                                 size_t errlen) {
    if (!json || !out) return -1;
    *out = nullptr;
    try {
        rmr_scene_blob* b = new rmr_scene_blob();
        if (variant == RMR_VARIANT_RM3 && len == 0) b->sc = rmr::builtin_scene(variant);
        else b->sc = rmr::compile_scene(std::string(json, len), variant);
        *out = b;
        return 0;
    } catch (const std::exception& e) {
        if (err && errlen) {
            std::snprintf(err, errlen, "%s", e.what());
        }
        return -3;
    }
}

extern "C" int rmr_scene_view(const rmr_scene_blob* b, rmr_scene* out) {
    if (!b || !out) return -1;
    *out = b->sc.view();
    return 0;
}

extern "C" void rmr_scene_free(rmr_scene_blob* b) { delete b; }
