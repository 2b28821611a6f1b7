"""oracle/glsl_ref/shader_build.py — TEST INFRASTRUCTURE: assemble a runnable copy of the
reference GLSL (read from /root/reference at run time; the output goes to oracle/_ref/, which is
git-ignored — reference source never enters the repo).

It restates Graphics::loadShader's marker expansion (Graphics.cpp:60-113) with the code generators
that feed it: v1 (Graphics.cpp:513-703, the producer of RayMarch.glsl's //#OBJINSERT,
//#OBJFUNCINSERT, //#MATFUNCINSERT, //#CASEINSERT bodies) and v2 (Graphics.cpp:392-509, 705-739,
RayMarch2.glsl's mat_func_1). Patches needed to compile/run on Mesa llvmpipe:
  P1  texture2D( -> texture(          (dead env-map branch; rejected under #version 430 core)
  P2  RayMarch2 struct member functions -> free functions (an NVIDIA-only GLSL extension)
  P3  zero-initialise generated out params / locals (`out` params are undefined on entry; rmr
      defines them as vec3(0))
  P4  (probe shaders only) main() renamed ref_main(); a KAT main() appended.
  X1  scenes with a map_mandelbulb node (not in the reference's node set) get the
      builder's GLSL statement of that node (EXT_MANDELBULB below, written for this harness, not
      taken from the reference) inserted with the object functions, in the reference's node ABI
      (vec3 in/out). It uses the driver's own pow/acos/atan/sin/cos/log, so the C3 fixture is
      "the reference path with that node added" (SURVEY §8d), pinned by PSNR like the others.
"""
import json
import os
import re

REF = "/root/reference/RayMarch Renderer"
SHADERS = {1: "RayMarch.glsl", 2: "RayMarch2.glsl", 3: "RayMarch3.glsl"}
LOCAL = {1: (8, 8), 2: (16, 16), 3: (16, 16)}


def _f(x):  # std::to_string(float(x)) == "%f"
    import struct
    return "%f" % struct.unpack("f", struct.pack("f", float(x)))[0]


def _jstr(x):  # jsoncpp asString() of a number (exact float round trip is what matters)
    return repr(float(x)) if not isinstance(x, int) else str(x)


def v1_objects(objects):
    """obj_func_<i> bodies, Graphics.cpp:647-702."""
    lines = []
    for i, obj in enumerate(objects):
        lines.append("void obj_func_%d(in vec3 p, out vec3 d)" % i)
        lines.append("{")
        tv = obj["total_vars"]
        lines.append("vec3 vars[%s];" % tv)
        lines.append("for (int zi = 0; zi < %s; zi++) vars[zi] = vec3(0);" % tv)  # P3
        for n in obj["nodes"]:
            s = n["name"] + "("
            for a in n["inputs"]:
                if isinstance(a, list):
                    a = list(a) + [0, 0, 0]
                    s += "vec3(%s, %s, %s), " % (_f(a[0]), _f(a[1]), _f(a[2]))
                elif a == -1:
                    s += "p, "
                else:
                    s += "vars[%d], " % a
            s += ", ".join("vars[%d]" % o for o in n["outputs"])
            s += ");"
            lines.append(s)
        lines.append("d = vars[%d];" % obj["distance"])
        lines.append("}")
    return lines


def v1_materials(materials):
    """mat_func_<id> bodies, Graphics.cpp:515-645."""
    lines = []
    for m in materials:
        lines.append("void mat_func_%d(inout RayData ray, out vec3 outColor, out vec3 outDir, "
                     "out vec3 outInside, out vec3 outHit)" % m["id"])
        lines.append("{")
        lines.append("outColor = vec3(0); outDir = vec3(0); outInside = vec3(0); outHit = vec3(0);")  # P3
        tv = m["total_vars"]
        lines.append("vec3 vars[%s];" % tv)
        lines.append("for (int zi = 0; zi < %s; zi++) vars[zi] = vec3(0);" % tv)  # P3
        names = {}
        for n in m["nodes"]:
            s = n["name"] + "(ray, "
            for a in n["inputs"]:
                if isinstance(a, list):
                    a = list(a) + [0, 0, 0]
                    s += "vec3(%s, %s, %s), " % (_f(a[0]), _f(a[1]), _f(a[2]))
                elif isinstance(a, str):
                    if a in names:
                        s += "vars[%d], " % names[a]
                elif isinstance(a, int):
                    s += "vars[%d], " % a
            outs = []
            for o in n["outputs"]:
                if isinstance(o, str):
                    if o not in names:
                        names[o] = len(names)
                    outs.append("vars[%d]" % names[o])
                elif isinstance(o, int):
                    outs.append("vars[%d]" % o)
            s += ", ".join(outs) + ");"
            lines.append(s)
        for key, out in (("color", "outColor"), ("dir", "outDir"), ("inside", "outInside"), ("hit", "outHit")):
            v = m.get(key)
            if isinstance(v, str):
                lines.append("%s = vars[%d];" % (out, names.get(v, 0)))
            elif isinstance(v, int) and not isinstance(v, bool) and v != -1:
                lines.append("%s = vars[%d];" % (out, v))
        lines.append("}")
    return lines


def v2_materials(materials):
    """mat_func_<id> for RayMarch2.glsl, Graphics.cpp:705-739 with compileNode 412-463."""
    lines = []

    def get_input(m, inp):
        c = m["constants"][inp[1]]
        if isinstance(c, list):
            return "vec3(%s, %s, %s)" % (_jstr(c[0]), _jstr(c[1]), _jstr(c[2]))
        return _jstr(c)

    def node(m, idx, o0, o1):
        n = m["nodes"][idx]
        name = n["name"]
        ins = n.get("inputs", [])
        if name == "shader_diffuse":
            lines.append(o0 + " = point.tbn * material_diffuse.samplePDF(point.dir);")
            lines.append(o1 + " = material_diffuse.weightPDF(point.dir, " + get_input(m, ins[0]) + ");")
        elif name == "shader_glossy":
            lines.append(o0 + " = point.tbn * material_glossy.samplePDF(point.dir, point.normal, " + get_input(m, ins[1]) + ");")
            lines.append(o1 + " = material_glossy.weightPDF(point.dir, vec3(" + get_input(m, ins[0]) + "));")
        elif name == "shader_mix":
            lines.append("vec3 " + o0 + "_mixDir[2];")
            lines.append("vec3 " + o0 + "_mixRefl[2];")
            lines.append("float " + o0 + "_mixFact;")
            lines.append(o0 + "_mixDir[0] = vec3(0); " + o0 + "_mixDir[1] = vec3(0); " + o0 + "_mixRefl[0] = vec3(0); "
                         + o0 + "_mixRefl[1] = vec3(0); " + o0 + "_mixFact = 0.0;")  # P3
            if ins[0][0] != -1:
                node(m, ins[0][0], o0 + "_mixDir[0]", o0 + "_mixRefl[0]")
            if ins[1][0] != -1:
                node(m, ins[1][0], o0 + "_mixDir[1]", o0 + "_mixRefl[1]")
            if ins[2][0] != -1:
                node(m, ins[2][0], o0 + "_mixFact", "")
            lines.append("float r = rand(point.pos.xz);")
            lines.append("if (r <= " + o0 + "_mixFact)")
            lines.append("{")
            lines.append(o0 + " = " + o0 + "_mixDir[1];")
            lines.append(o1 + " = " + o0 + "_mixRefl[1];")
            lines.append("}")
            lines.append("else")
            lines.append("{")
            lines.append(o0 + " = " + o0 + "_mixDir[0];")
            lines.append(o1 + " = " + o0 + "_mixRefl[0];")
            lines.append("}")
        elif name == "misc_fresnel":
            lines.append(o0 + " = pow(1.0 - clamp(dot(point.normal, point.dir), 0.0, 1.0), 5) * 0.96 + 0.04;")

    for m in materials:
        lines += ["void mat_func_%d(in PointData point, in vec3 color, out MatData matData)" % m["id"], "{",
                  "MatData mat;", "mat.color = color;", "mat.light = vec3(0);", "mat.newDir = vec3(0);",
                  "mat.willBreak = false;", "vec3 reflectance = vec3(0);", "vec3 newDir = vec3(0);"]  # P3
        node(m, m["output"], "newDir", "reflectance")
        lines += ["mat.newDir = newDir;",
                  "float probability = max(reflectance.r, max(reflectance.g, reflectance.b));",
                  "if (rand(point.pos.zx) <= 1)", "{", "\tmat.color *= reflectance / probability;",
                  "\tmat.willBreak = false;", "}", "else", "{", "\tmat.willBreak = true;", "}",
                  "matData = mat;", "}"]
    return lines


# X1: the Mandelbulb distance estimator as a v1 object node (same statement as rmr's sd_mandelbulb:
# csrc/rmr_trace.h; inputs P, centre, (power, iterations, bailout))
EXT_MANDELBULB = r"""
void map_mandelbulb(in vec3 p, in vec3 centre, in vec3 prm, out vec3 d)
{
	vec3 p0 = p - centre;
	vec3 z = p0;
	float power = prm.x;
	float bail = prm.z;
	int iters = int(prm.y);
	float dr = 1.0;
	float r = 0.0;
	for (int i = 0; i < iters; i++)
	{
		r = length(z);
		if (r > bail) break;
		float theta = acos(z.z / r);
		float phi = atan(z.y, z.x);
		dr = pow(r, power - 1.0) * power * dr + 1.0;
		float zr = pow(r, power);
		theta = theta * power;
		phi = phi * power;
		z = vec3(sin(theta) * cos(phi), sin(phi) * sin(theta), cos(theta)) * zr + p0;
	}
	d = vec3(0.5 * log(r) * r / dr);
}  // (not a bare "}": expand() counts objects by those lines)
"""


def _uses(objects, name):
    return any(n.get("name") == name for o in objects for n in o.get("nodes", []))


def expand(src_lines, mat_lines, obj_lines, objects):
    """Graphics::loadShader marker expansion, Graphics.cpp:60-113."""
    lines = list(src_lines)
    i = 0
    while i < len(lines):
        line = lines[i]
        if "//#MATFUNCINSERT" in line:
            lines[i:i + 1] = mat_lines
        elif "//#CASEINSERT" in line:
            mat_num = sum(1 for l in mat_lines if l == "}")
            ins = []
            for j in range(mat_num):
                ins += ["\t\t\tcase %d:" % j, "\t\t\t\tmat_func_%d(ray, newColor, newDir, newInside, newHit);" % j,
                        "\t\t\t\tbreak;"]
            lines[i:i + 1] = ins
        elif "//#OBJFUNCINSERT" in line:
            lines[i:i + 1] = obj_lines
        elif "//#OBJINSERT" in line:
            obj_num = sum(1 for l in obj_lines if l == "}")
            ins = []
            for j in range(obj_num):
                ins += ["\tvec3 d%d;" % j, "\tobj_func_%d(p, d%d);" % (j, j),
                        "\td = opU(d, vec2(d%d.x, %d));" % (j, objects[j].get("matID", 0))]
            lines[i:i + 1] = ins
        i += 1
    return lines


def _struct_to_functions(src, struct_name, inst):  # P2
    m = re.search(r"struct\s+%s\s*(//[^\n]*)?\s*\{" % struct_name, src)
    if not m:
        return src
    start = m.end() - 1
    depth = 0
    for k in range(start, len(src)):
        if src[k] == "{":
            depth += 1
        elif src[k] == "}":
            depth -= 1
            if depth == 0:
                end = k
                break
    body = src[start + 1:end]
    tail = re.match(r"\}\s*%s\s*;" % inst, src[end:])
    body = re.sub(r"\bvec3\s+(brdf|samplePDF|weightPDF)\s*\(", lambda mm: "vec3 %s_%s(" % (inst, mm.group(1)), body)
    return src[:m.start()] + body + src[end + tail.end():]


def build(variant, scene=None, probe_main=None):
    """Returns GLSL source text for variant 1/2/3 with `scene` (dict) compiled in."""
    with open(os.path.join(REF, SHADERS[variant]), "r") as f:
        src = f.read()
    src = src.replace("texture2D(", "texture(")  # P1
    scene = scene or {}
    if variant == 1:
        mat_lines = v1_materials(scene.get("materials", []))
        obj_lines = v1_objects(scene.get("objects", []))
        if _uses(scene.get("objects", []), "map_mandelbulb"):   # X1 (not a reference node)
            obj_lines = EXT_MANDELBULB.strip("\n").split("\n") + obj_lines
    elif variant == 2:
        mat_lines = v2_materials(scene.get("materials", []))
        obj_lines = []
    else:
        mat_lines, obj_lines = [], []
    lines = expand(src.split("\n"), mat_lines, obj_lines, scene.get("objects", []))
    src = "\n".join(lines)
    if variant == 2:
        src = _struct_to_functions(src, "DiffuseMaterial", "material_diffuse")
        src = _struct_to_functions(src, "GlossyMaterial", "material_glossy")
        src = src.replace("material_diffuse.", "material_diffuse_").replace("material_glossy.", "material_glossy_")
        src = src.replace("vec3 matColor;", "vec3 matColor = vec3(0);")  # P3 (ids without a case)
    if variant == 3:
        src = src.replace("vec3 newDir;", "vec3 newDir = vec3(0);")  # P3 (ids without a branch)
    if probe_main is not None:  # P4
        src = re.sub(r"\bvoid\s+main\s*\(\s*\)", "void ref_main()", src)
        src += "\n" + probe_main + "\n"
    return src


def load_scene(path):
    with open(path, "r") as f:
        return json.load(f)
