/*
 * oracle/glsl_ref/harness.c — TEST INFRASTRUCTURE: runs the reference's GLSL compute shaders
 * (RayMarch*.glsl, read from /root/reference at run time, never copied into the repo) headless on
 * Mesa llvmpipe through the DRI swrast driver interface (no X / EGL / OSMesa needed).
 *
 * It plays the role of Graphics::Render (Graphics.cpp:314-354): same uniforms, image unit 0 =
 * RGBA32F accumulator, unit 1 = the 1x1 materialData texture; one glDispatchCompute per
 * (time, currentSample, bounds) line, followed by glMemoryBarrier (the reference has none).
 *
 * usage: harness <shader.glsl> <job.txt> <out_image.f32> [out_ssbo.f32]
 * job.txt lines:
 *   image W H                      RGBA32F accumulator (cleared to 0)
 *   uf NAME v | ui NAME v | u3f NAME x y z | u4f NAME x y z w
 *   ssbo_in PATH                   float buffer at binding 2 (probe shaders)
 *   ssbo_out N                     float buffer of N floats at binding 3, written to out_ssbo
 *   run TIME SAMPLE BX0 BY0 BX1 BY1 GX GY    set time/currentSample/bounds, dispatch GXxGYx1
 */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <GL/glcorearb.h>
#include <GL/internal/dri_interface.h>

static void gdi(__DRIdrawable* d, int* x, int* y, int* w, int* h, void* p) { (void)d; (void)p; *x = 0; *y = 0; *w = 1; *h = 1; }
static void pim(__DRIdrawable* d, int op, int x, int y, int w, int h, char* data, void* p) {
    (void)d; (void)op; (void)x; (void)y; (void)w; (void)h; (void)data; (void)p;
}
static void gim(__DRIdrawable* d, int x, int y, int w, int h, char* data, void* p) {
    (void)d; (void)x; (void)y; (void)w; (void)h; (void)data; (void)p;
}
static const __DRIswrastLoaderExtension loader = {{__DRI_SWRAST_LOADER, 1}, gdi, pim, gim, NULL, NULL};
static const __DRIextension* loader_exts[] = {&loader.base, NULL};

typedef void* (*getproc_t)(const char*);
static getproc_t getproc;
#define GLF(type, name) static type p_##name;
GLF(PFNGLCREATESHADERPROC, glCreateShader)
GLF(PFNGLSHADERSOURCEPROC, glShaderSource)
GLF(PFNGLCOMPILESHADERPROC, glCompileShader)
GLF(PFNGLGETSHADERIVPROC, glGetShaderiv)
GLF(PFNGLGETSHADERINFOLOGPROC, glGetShaderInfoLog)
GLF(PFNGLCREATEPROGRAMPROC, glCreateProgram)
GLF(PFNGLATTACHSHADERPROC, glAttachShader)
GLF(PFNGLLINKPROGRAMPROC, glLinkProgram)
GLF(PFNGLGETPROGRAMIVPROC, glGetProgramiv)
GLF(PFNGLGETPROGRAMINFOLOGPROC, glGetProgramInfoLog)
GLF(PFNGLUSEPROGRAMPROC, glUseProgram)
GLF(PFNGLGETUNIFORMLOCATIONPROC, glGetUniformLocation)
GLF(PFNGLUNIFORM1FPROC, glUniform1f)
GLF(PFNGLUNIFORM1IPROC, glUniform1i)
GLF(PFNGLUNIFORM3FPROC, glUniform3f)
GLF(PFNGLUNIFORM4FPROC, glUniform4f)
GLF(PFNGLGENTEXTURESPROC, glGenTextures)
GLF(PFNGLBINDTEXTUREPROC, glBindTexture)
GLF(PFNGLACTIVETEXTUREPROC, glActiveTexture)
GLF(PFNGLTEXIMAGE2DPROC, glTexImage2D)
GLF(PFNGLTEXPARAMETERIPROC, glTexParameteri)
GLF(PFNGLBINDIMAGETEXTUREPROC, glBindImageTexture)
GLF(PFNGLDISPATCHCOMPUTEPROC, glDispatchCompute)
GLF(PFNGLMEMORYBARRIERPROC, glMemoryBarrier)
GLF(PFNGLFINISHPROC, glFinish)
GLF(PFNGLGETTEXIMAGEPROC, glGetTexImage)
GLF(PFNGLGETSTRINGPROC, glGetString)
GLF(PFNGLGENBUFFERSPROC, glGenBuffers)
GLF(PFNGLBINDBUFFERPROC, glBindBuffer)
GLF(PFNGLBUFFERDATAPROC, glBufferData)
GLF(PFNGLBINDBUFFERBASEPROC, glBindBufferBase)
GLF(PFNGLGETBUFFERSUBDATAPROC, glGetBufferSubData)
GLF(PFNGLGETERRORPROC, glGetError)
#define LOAD(name)                                                         \
    do {                                                                   \
        p_##name = (void*)getproc(#name);                                  \
        if (!p_##name) { fprintf(stderr, "missing %s\n", #name); exit(3); } \
    } while (0)

static char* slurp(const char* path, long* n) {
    FILE* f = fopen(path, "rb");
    if (!f) { perror(path); exit(2); }
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    char* b = malloc(sz + 1);
    if (fread(b, 1, sz, f) != (size_t)sz) { perror("read"); exit(2); }
    b[sz] = 0;
    fclose(f);
    if (n) *n = sz;
    return b;
}

int main(int argc, char** argv) {
    if (argc < 4) { fprintf(stderr, "usage: harness shader job out [ssbo_out]\n"); return 1; }
    void* glapi = dlopen("libglapi.so.0", RTLD_NOW | RTLD_GLOBAL);
    if (!glapi) { fprintf(stderr, "dlopen libglapi: %s\n", dlerror()); return 2; }
    const char* drvpath = getenv("RMR_SWRAST") ? getenv("RMR_SWRAST") : "/usr/lib/x86_64-linux-gnu/dri/swrast_dri.so";
    void* drv = dlopen(drvpath, RTLD_NOW | RTLD_GLOBAL);
    if (!drv) { fprintf(stderr, "dlopen swrast: %s\n", dlerror()); return 2; }
    const __DRIextension** (*getext)(void) = (const __DRIextension** (*)(void))dlsym(drv, "__driDriverGetExtensions_swrast");
    getproc = (getproc_t)dlsym(glapi, "_glapi_get_proc_address");
    if (!getext || !getproc) { fprintf(stderr, "missing driver entry points\n"); return 2; }
    const __DRIextension** ext = getext();
    const __DRIcoreExtension* core = NULL;
    const __DRIswrastExtension* sw = NULL;
    for (int i = 0; ext[i]; i++) {
        if (!strcmp(ext[i]->name, __DRI_CORE)) core = (const __DRIcoreExtension*)ext[i];
        if (!strcmp(ext[i]->name, __DRI_SWRAST)) sw = (const __DRIswrastExtension*)ext[i];
    }
    if (!core || !sw || sw->base.version < 4) { fprintf(stderr, "no DRI core/swrast v4\n"); return 2; }
    const __DRIconfig** cfgs = NULL;
    __DRIscreen* scr = sw->createNewScreen2(0, loader_exts, ext, &cfgs, NULL);
    if (!scr || !cfgs || !cfgs[0]) { fprintf(stderr, "createNewScreen2 failed\n"); return 2; }
    uint32_t attribs[] = {__DRI_CTX_ATTRIB_MAJOR_VERSION, 4, __DRI_CTX_ATTRIB_MINOR_VERSION, 3};
    unsigned err = 0;
    __DRIcontext* ctx = sw->createContextAttribs(scr, __DRI_API_OPENGL_CORE, cfgs[0], NULL, 2, attribs, &err, NULL);
    if (!ctx) { fprintf(stderr, "createContextAttribs failed (%u)\n", err); return 2; }
    if (!core->bindContext(ctx, NULL, NULL)) { fprintf(stderr, "bindContext failed\n"); return 2; }
    LOAD(glCreateShader); LOAD(glShaderSource); LOAD(glCompileShader); LOAD(glGetShaderiv);
    LOAD(glGetShaderInfoLog); LOAD(glCreateProgram); LOAD(glAttachShader); LOAD(glLinkProgram);
    LOAD(glGetProgramiv); LOAD(glGetProgramInfoLog); LOAD(glUseProgram); LOAD(glGetUniformLocation);
    LOAD(glUniform1f); LOAD(glUniform1i); LOAD(glUniform3f); LOAD(glUniform4f); LOAD(glGenTextures);
    LOAD(glBindTexture); LOAD(glActiveTexture); LOAD(glTexImage2D); LOAD(glTexParameteri); LOAD(glBindImageTexture);
    LOAD(glDispatchCompute); LOAD(glMemoryBarrier); LOAD(glFinish); LOAD(glGetTexImage);
    LOAD(glGetString); LOAD(glGenBuffers); LOAD(glBindBuffer); LOAD(glBufferData);
    LOAD(glBindBufferBase); LOAD(glGetBufferSubData); LOAD(glGetError);
    if (getenv("RMR_VERBOSE")) fprintf(stderr, "GL_VERSION %s\n", (const char*)p_glGetString(GL_VERSION));

    const char* src = slurp(argv[1], NULL);
    GLuint sh = p_glCreateShader(GL_COMPUTE_SHADER);
    p_glShaderSource(sh, 1, &src, NULL);
    p_glCompileShader(sh);
    GLint ok = 0;
    p_glGetShaderiv(sh, GL_COMPILE_STATUS, &ok);
    if (!ok) {
        static char log[65536];
        p_glGetShaderInfoLog(sh, sizeof log, NULL, log);
        fprintf(stderr, "COMPILE ERROR\n%s\n", log);
        return 4;
    }
    GLuint prog = p_glCreateProgram();
    p_glAttachShader(prog, sh);
    p_glLinkProgram(prog);
    p_glGetProgramiv(prog, GL_LINK_STATUS, &ok);
    if (!ok) {
        static char log[65536];
        p_glGetProgramInfoLog(prog, sizeof log, NULL, log);
        fprintf(stderr, "LINK ERROR\n%s\n", log);
        return 4;
    }
    p_glUseProgram(prog);

    int W = 0, H = 0;
    GLuint tex = 0, mtex = 0, sin_buf = 0, sout_buf = 0;
    long sout_n = 0;
    char* job = slurp(argv[2], NULL);
    for (char* line = strtok(job, "\n"); line; line = strtok(NULL, "\n")) {
        char name[128];
        float a, b, c, d;
        int i0, ew, eh;
        if (sscanf(line, "image %d %d", &W, &H) == 2) {
            float* zero = calloc((size_t)W * H * 4, sizeof(float));
            p_glGenTextures(1, &tex);
            p_glBindTexture(GL_TEXTURE_2D, tex);
            p_glTexImage2D(GL_TEXTURE_2D, 0, GL_RGBA32F, W, H, 0, GL_RGBA, GL_FLOAT, zero);
            p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MIN_FILTER, GL_NEAREST);
            p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MAG_FILTER, GL_NEAREST);
            p_glBindImageTexture(0, tex, 0, GL_FALSE, 0, GL_READ_WRITE, GL_RGBA32F);
            float one[4] = {0, 0, 0, 0};
            p_glGenTextures(1, &mtex);
            p_glBindTexture(GL_TEXTURE_2D, mtex);
            p_glTexImage2D(GL_TEXTURE_2D, 0, GL_RGBA32F, 1, 1, 0, GL_RGBA, GL_FLOAT, one);
            p_glBindImageTexture(1, mtex, 0, GL_FALSE, 0, GL_READ_WRITE, GL_RGBA32F);
            free(zero);
        } else if (sscanf(line, "envtex %127s %d %d", name, &ew, &eh) == 3) {
            /* envTex sampler (texture unit 0): RGBA8, bilinear, clamp to edge, no mipmaps */
            long n = 0;
            char* data = slurp(name, &n);
            if (n != (long)ew * eh * 4) { fprintf(stderr, "envtex size mismatch\n"); return 1; }
            GLuint et = 0;
            p_glActiveTexture(GL_TEXTURE0);
            p_glGenTextures(1, &et);
            p_glBindTexture(GL_TEXTURE_2D, et);
            p_glTexImage2D(GL_TEXTURE_2D, 0, GL_RGBA8, ew, eh, 0, GL_RGBA, GL_UNSIGNED_BYTE, data);
            p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MIN_FILTER, GL_LINEAR);
            p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MAG_FILTER, GL_LINEAR);
            p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_WRAP_S, GL_CLAMP_TO_EDGE);
            p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_WRAP_T, GL_CLAMP_TO_EDGE);
            free(data);
        } else if (sscanf(line, "uf %127s %f", name, &a) == 2) {
            p_glUniform1f(p_glGetUniformLocation(prog, name), a);
        } else if (sscanf(line, "ui %127s %d", name, &i0) == 2) {
            p_glUniform1i(p_glGetUniformLocation(prog, name), i0);
        } else if (sscanf(line, "u3f %127s %f %f %f", name, &a, &b, &c) == 4) {
            p_glUniform3f(p_glGetUniformLocation(prog, name), a, b, c);
        } else if (sscanf(line, "u4f %127s %f %f %f %f", name, &a, &b, &c, &d) == 5) {
            p_glUniform4f(p_glGetUniformLocation(prog, name), a, b, c, d);
        } else if (sscanf(line, "ssbo_in %127s", name) == 1) {
            long n = 0;
            char* data = slurp(name, &n);
            p_glGenBuffers(1, &sin_buf);
            p_glBindBuffer(GL_SHADER_STORAGE_BUFFER, sin_buf);
            p_glBufferData(GL_SHADER_STORAGE_BUFFER, n, data, GL_STATIC_DRAW);
            p_glBindBufferBase(GL_SHADER_STORAGE_BUFFER, 2, sin_buf);
            free(data);
        } else if (sscanf(line, "ssbo_out %ld", &sout_n) == 1) {
            p_glGenBuffers(1, &sout_buf);
            p_glBindBuffer(GL_SHADER_STORAGE_BUFFER, sout_buf);
            p_glBufferData(GL_SHADER_STORAGE_BUFFER, sout_n * 4, NULL, GL_DYNAMIC_READ);
            p_glBindBufferBase(GL_SHADER_STORAGE_BUFFER, 3, sout_buf);
        } else if (strncmp(line, "run ", 4) == 0) {
            float t, bx0, by0, bx1, by1;
            int smp, ngx, ngy;
            if (sscanf(line + 4, "%f %d %f %f %f %f %d %d", &t, &smp, &bx0, &by0, &bx1, &by1, &ngx, &ngy) != 8) {
                fprintf(stderr, "bad run line: %s\n", line);
                return 1;
            }
            p_glUniform1f(p_glGetUniformLocation(prog, "time"), t);
            p_glUniform1i(p_glGetUniformLocation(prog, "currentSample"), smp);
            p_glUniform4f(p_glGetUniformLocation(prog, "bounds"), bx0, by0, bx1, by1);
            p_glDispatchCompute((GLuint)ngx, (GLuint)ngy, 1);
            p_glMemoryBarrier(GL_ALL_BARRIER_BITS);
        }
    }
    p_glFinish();
    GLenum e = p_glGetError();
    if (e != GL_NO_ERROR) { fprintf(stderr, "GL error 0x%x\n", e); return 5; }
    FILE* f = fopen(argv[3], "wb");
    if (tex) {
        float* img = malloc((size_t)W * H * 4 * sizeof(float));
        p_glBindTexture(GL_TEXTURE_2D, tex);
        p_glGetTexImage(GL_TEXTURE_2D, 0, GL_RGBA, GL_FLOAT, img);
        fwrite(img, sizeof(float), (size_t)W * H * 4, f);
        free(img);
    }
    fclose(f);
    if (sout_buf && argc > 4) {
        float* out = malloc(sout_n * 4);
        p_glBindBuffer(GL_SHADER_STORAGE_BUFFER, sout_buf);
        p_glGetBufferSubData(GL_SHADER_STORAGE_BUFFER, 0, sout_n * 4, out);
        FILE* g = fopen(argv[4], "wb");
        fwrite(out, 4, sout_n, g);
        fclose(g);
        free(out);
    }
    return 0;
}
