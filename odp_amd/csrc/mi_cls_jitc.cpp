// mi_cls_jitc: compiles one program-specialised classification kernel with
// hipRTC in a process of its own (libmi_cls.so starts it, mi_cls.hip
// spec_compile).  Compiling in the library's own process left a compiler
// thread running when a short-lived process exited, and the exit-time
// teardown could deadlock with it; a child process holds nothing the parent
// tears down, and the parent kills it at exit instead of waiting.
//
// Protocol (stdin): four length-prefixed sections, each "<bytes>\n" then the
// bytes -- the kernel source, mi_cls.h, mi_cls_dev.h, and the name
// expression of the kernel instantiation; argv[1..] are the compile options.
// stdout on success: "OK <lowered-name-bytes> <code-bytes>\n", the lowered
// name, the code object.  On failure: "ERR <log-bytes>\n" and the log.
// Exit status 0 either way when the protocol held, 2 on a malformed input.
#include <hip/hiprtc.h>

#include <stdio.h>
#include <stdlib.h>
#include <string>
#include <vector>

static bool read_section(std::string &out)
{
	unsigned long n = 0;
	if (scanf("%lu", &n) != 1 || getchar() != '\n' || n > (64ul << 20))
		return false;
	out.resize(n);
	return n == 0 || fread(&out[0], 1, n, stdin) == n;
}

int main(int argc, char **argv)
{
	std::string src, h, dev, name;
	if (!read_section(src) || !read_section(h) || !read_section(dev) || !read_section(name))
		return 2;
	const char *hdrs[2] = { h.c_str(), dev.c_str() };
	const char *names[2] = { "mi_cls.h", "mi_cls_dev.h" };
	std::string log;
	hiprtcProgram p;
	if (hiprtcCreateProgram(&p, src.c_str(), "mi_cls_spec.hip", 2, hdrs, names) != HIPRTC_SUCCESS) {
		printf("ERR 0\n");
		return 0;
	}
	std::vector<const char *> opts(argv + 1, argv + argc);
	hiprtcAddNameExpression(p, name.c_str());
	const hiprtcResult r = hiprtcCompileProgram(p, (int)opts.size(), opts.data());
	size_t ls = 0, cs = 0;
	if (hiprtcGetProgramLogSize(p, &ls) == HIPRTC_SUCCESS && ls > 1) {
		log.resize(ls);
		hiprtcGetProgramLog(p, &log[0]);
	}
	const char *ln = nullptr;
	std::vector<char> code;
	if (r == HIPRTC_SUCCESS && hiprtcGetCodeSize(p, &cs) == HIPRTC_SUCCESS && cs &&
	    hiprtcGetLoweredName(p, name.c_str(), &ln) == HIPRTC_SUCCESS && ln) {
		code.resize(cs);
		if (hiprtcGetCode(p, code.data()) == HIPRTC_SUCCESS) {
			const std::string low = ln;
			printf("OK %zu %zu\n", low.size(), code.size());
			fwrite(low.data(), 1, low.size(), stdout);
			fwrite(code.data(), 1, code.size(), stdout);
			fflush(stdout);
			hiprtcDestroyProgram(&p);
			return 0;
		}
	}
	printf("ERR %zu\n", log.size());
	fwrite(log.data(), 1, log.size(), stdout);
	fflush(stdout);
	hiprtcDestroyProgram(&p);
	return 0;
}
