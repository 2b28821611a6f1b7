/*
 * rmr_tables.h — plain-data scene tables consumed by the rmr ray-march path tracer.
 *
 * The reference (TheBinaryCodeX/RayMarchRenderer) turns its JSON scene files into GLSL *source text*
 * and recompiles the compute shader on every Graphics::Reload (Graphics.cpp:511-752, marker
 * expansion Graphics.cpp:60-113). rmr replaces that code generator with these tables: the host
 * compiles a scene once into prims / ops / constants / materials, and the HIP kernels interpret
 * them. Nothing here is a torch or HIP type; the same tables feed the C-ABI
 * (rmr_load_scene_tables) and the CPU oracle under oracle/.
 *
 * Layout notes:
 *   - rmr_prim     48 B, one per `objects[j]` in scene order (order matters: opU ties pick the later
 *                  object, RayMarch.glsl:219-222).
 *   - rmr_op       48 B, one node of an object SDF program or a v1/v2 material program.
 *   - consts       float[3] triples; literals are quantised exactly as the reference codegen
 *                  prints them (std::to_string(float) = "%f", Graphics.cpp:542,670).
 */
#ifndef RMR_TABLES_H
#define RMR_TABLES_H

#ifdef __HIPCC_RTC__ /* hipRTC (per-scene kernel specialisation) has no <stdint.h> */
typedef __hip_internal::int32_t int32_t;
typedef __hip_internal::uint32_t uint32_t;
typedef __hip_internal::int64_t int64_t;
typedef __hip_internal::uint64_t uint64_t;
typedef __hip_internal::uint8_t uint8_t;
#else
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* ---- limits ---------------------------------------------------------------------------- */
#define RMR_MAX_VARS      16   /* vec3 vars[total_vars] per generated function              */
#define RMR_MAX_PRIMS     4096
#define RMR_MAX_OPS       8192
#define RMR_MAX_CONSTS    8192
#define RMR_MAX_MATERIALS 256

/* ---- kernel variants (one per reference compute shader) -------------------------------- */
typedef enum rmr_variant {
    RMR_VARIANT_RM1 = 1, /* RayMarch.glsl  : node-graph RGB path tracer                       */
    RMR_VARIANT_RM2 = 2, /* RayMarch2.glsl : RGB + next-event estimation ("light-march")      */
    RMR_VARIANT_RM3 = 3  /* RayMarch3.glsl : spectral hero-wavelength path tracer (wired in)  */
} rmr_variant;

/* ---- primitives (one per scene object) -------------------------------------------------- */
typedef enum rmr_prim_type {
    RMR_PRIM_SPHERE     = 1, /* map_sphere(p, c, r)      RayMarch.glsl:170-174 (uses r.x)     */
    RMR_PRIM_BOX        = 2, /* map_box(p, c, r)         RayMarch.glsl:176-180                */
    RMR_PRIM_PROGRAM    = 3, /* generic obj_func_j node program (Graphics.cpp:648-702)        */
    RMR_PRIM_MANDELBULB = 4  /* new node: c = centre, r = {power, iters, bail}*/
} rmr_prim_type;

typedef struct rmr_prim {
    int32_t type;       /* rmr_prim_type                                                      */
    float   mat_id;     /* float(objects[j]["matID"]) — the map() vec2.y                      */
    int32_t prog_begin; /* PROGRAM: first op in ops[]                                         */
    int32_t prog_end;   /* PROGRAM: one past the last op                                      */
    float   c[3];       /* centre                                                             */
    int32_t dist_var;   /* PROGRAM: var holding the distance (objects[j]["distance"])         */
    float   r[3];       /* radius / half size / mandelbulb parameters                          */
    int32_t n_vars;     /* PROGRAM: total_vars                                                */
} rmr_prim;

/* ---- node ops ---------------------------------------------------------------------------- */
/* Operand encoding in rmr_op.in[]: >= 0 var index; RMR_OPND_P = the sample point p (object
 * programs only); <= RMR_OPND_CONST0 : constant index (RMR_OPND_CONST0 - k); RMR_OPND_NONE unused. */
#define RMR_OPND_NONE   (-1000000)
#define RMR_OPND_P      (-1)
#define RMR_OPND_CONST0 (-2)
#define RMR_OPND_IS_CONST(x) ((x) <= RMR_OPND_CONST0 && (x) > RMR_OPND_NONE)
#define RMR_OPND_CONST_INDEX(x) (RMR_OPND_CONST0 - (x))

typedef enum rmr_opcode {
    /* object (SDF) nodes, RayMarch.glsl:121-215 */
    RMR_OP_GET_X = 1, RMR_OP_GET_Y, RMR_OP_GET_Z,
    RMR_OP_ADD, RMR_OP_SUB, RMR_OP_MUL, RMR_OP_DIV, RMR_OP_SIN, RMR_OP_COS,
    RMR_OP_MAP_SPHERE, RMR_OP_MAP_BOX,
    RMR_OP_UNION, RMR_OP_SUBTRACT, RMR_OP_INTERSECT,
    RMR_OP_DOMAIN_REPEAT,
    RMR_OP_MAP_MANDELBULB,
    /* v1 material nodes, RayMarch.glsl:313-479 */
    RMR_OP_M_FACING = 32, RMR_OP_M_INSIDE,
    RMR_OP_M_ADD, RMR_OP_M_SUB, RMR_OP_M_MUL, RMR_OP_M_DIV,
    RMR_OP_M_MIX, RMR_OP_M_DIFFUSE, RMR_OP_M_GLOSSY, RMR_OP_M_REFRACTION,
    RMR_OP_M_VOLUME, RMR_OP_M_EMISSION,
    /* v2 material nodes (RayMarch2.glsl + Graphics.cpp:412-463); slots are vec3 (fact in .x)  */
    RMR_OP_V2_DIFFUSE = 64, /* in[0]=const color            out[0]=dir slot out[1]=refl slot */
    RMR_OP_V2_GLOSSY,       /* in[0]=const color in[1]=const roughness (.x) out dir, refl     */
    RMR_OP_V2_FRESNEL,      /* out[0]=fact slot                                               */
    RMR_OP_V2_MIX           /* in: dir0 refl0 dir1 refl1 fact (slots)  out[0]=dir out[1]=refl */
} rmr_opcode;

typedef struct rmr_op {
    int32_t code;
    int32_t in[7];
    int32_t out[4];
} rmr_op;

/* ---- materials --------------------------------------------------------------------------- */
/* RM1 (v1 format): mat_func_<j>(ray, outColor, outDir, outInside, outHit) for case j. */
typedef struct rmr_material {
    int32_t defined;     /* 1 if `case j:` exists                                            */
    int32_t prog_begin, prog_end;
    int32_t n_vars;      /* total_vars                                                        */
    int32_t color_var;   /* var index or -1 = "not written" (stays vec3(0), App. A.5)         */
    int32_t dir_var;
    int32_t inside_var;
    int32_t hit_var;
} rmr_material;

/* RM3 spectral material (RayMarch3.glsl:251-345 mat_func_0..2, sky 408-438). */
typedef struct rmr_spectral {
    int32_t defined;
    uint32_t min_wave, max_wave; /* nm, band is inclusive                                    */
    float   power;               /* throughput multiplier                                     */
    int32_t terminates;          /* 1 = emitter: path always ends after the event (id 0)      */
    int32_t pad[3];
} rmr_spectral;

/* RM2 fixed-function diffuse albedo table (RayMarch2.glsl:445-456) + point light. */
typedef struct rmr_rm2_consts {
    float albedo[RMR_MAX_MATERIALS][3]; /* ids without a case stay 0                          */
    float light_pos[3];                 /* (2, 6, -2)  RayMarch2.glsl:458                      */
    float light_power;                  /* 50          RayMarch2.glsl:459                      */
    int32_t node_mat_id;                /* id dispatched to the generated mat_func (1)        */
    int32_t pad[3];
} rmr_rm2_consts;

/* ---- a compiled scene -------------------------------------------------------------------- */
typedef struct rmr_scene {
    int32_t variant;               /* rmr_variant                                             */
    int32_t n_prims;
    const rmr_prim* prims;
    int32_t n_ops;
    const rmr_op* ops;
    int32_t n_consts;
    const float* consts;           /* n_consts * 3                                            */
    int32_t n_materials;           /* RM1: number of cases; RM3: spectral entries              */
    const rmr_material* materials; /* RM1                                                     */
    const rmr_spectral* spectral;  /* RM3: [n_materials]                                      */
    rmr_spectral spectral_sky;     /* RM3 sky band                                            */
    int32_t v2_prog_begin, v2_prog_end; /* RM2: flattened mat_func_<node_mat_id>             */
    int32_t v2_n_slots;
    const rmr_rm2_consts* rm2;     /* RM2                                                     */
    float sky[3];                  /* skyColor(): vec3(0.015) (useEnvTex = 0, Graphics.cpp:338) */
} rmr_scene;

#ifdef __cplusplus
}
#endif
#endif /* RMR_TABLES_H */
