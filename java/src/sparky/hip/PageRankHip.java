// Java 22+ Panama FFM binding of libpagerank_hip (include/pagerank_hip.h) -- the north-star host.
//
// Binds exactly the C ABI the drop-in needs: pr_graph_create (Sparky.java:124-184), pr_run with
// a per-iteration upcall (Sparky.java:164-238, :188, :237), pr_graph_info, pr_last_error,
// pr_graph_destroy.  Non-zero status -> RuntimeException(pr_last_error()), as INTEGRATION.md
// specifies.  Host arrays are copied into a confined arena for the call only (the ABI borrows
// them); device memory belongs to the library.
//
// Build: java/Makefile (javac --release 22).  No JDK exists in the image this repository is
// developed in, so this file is compiled only where one does (tests/test_java_host.py checks the
// symbols it binds against the headers everywhere).
package sparky.hip;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_DOUBLE;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

import java.lang.foreign.Arena;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.SymbolLookup;
import java.lang.invoke.MethodHandle;
import java.lang.invoke.MethodHandles;
import java.lang.invoke.MethodType;

public final class PageRankHip implements AutoCloseable {
    /** pr_graph_create flags (include/pagerank_hip.h). */
    public static final int PR_DANGLING_LOCAL = 0, PR_DANGLING_NONE = 1, PR_NO_CANONICAL = 4;
    static final int PR_CB_RANKS = 1;
    static final int PR_INFO_COUNT = 24;
    /** PR_ABI_VERSION of include/pagerank_hip.h this binding was written against. */
    public static final int ABI_VERSION = 2;

    private static final Linker LINKER = Linker.nativeLinker();
    private static final SymbolLookup LIB = SymbolLookup.libraryLookup(
            System.getProperty("pagerank.hip.lib", "libpagerank_hip.so"), Arena.global());

    private static MethodHandle h(String name, FunctionDescriptor d) {
        return LINKER.downcallHandle(LIB.find(name).orElseThrow(
                () -> new UnsatisfiedLinkError("libpagerank_hip lacks " + name)), d);
    }

    private static final MethodHandle CREATE = h("pr_graph_create", FunctionDescriptor.of(JAVA_INT,
            JAVA_INT, JAVA_INT, JAVA_LONG, ADDRESS, ADDRESS, JAVA_INT, ADDRESS));
    private static final MethodHandle RUN = h("pr_run", FunctionDescriptor.of(JAVA_INT,
            ADDRESS, JAVA_INT, JAVA_DOUBLE, JAVA_DOUBLE, ADDRESS, ADDRESS, ADDRESS, JAVA_INT, ADDRESS));
    private static final MethodHandle INFO = h("pr_graph_info", FunctionDescriptor.of(JAVA_INT,
            ADDRESS, ADDRESS, JAVA_INT));
    private static final MethodHandle DESTROY = h("pr_graph_destroy", FunctionDescriptor.ofVoid(ADDRESS));
    private static final MethodHandle LAST_ERROR = h("pr_last_error", FunctionDescriptor.of(ADDRESS));
    private static final MethodHandle ABI = h("pr_abi_version", FunctionDescriptor.of(JAVA_INT));

    static {
        try {
            int v = (int) ABI.invokeExact();
            if (v != ABI_VERSION)
                throw new UnsatisfiedLinkError("libpagerank_hip ABI " + v + ", this binding needs " + ABI_VERSION);
        } catch (UnsatisfiedLinkError e) {
            throw e;
        } catch (Throwable t) {
            throw new ExceptionInInitializerError(t);
        }
    }
    private static final FunctionDescriptor CB_DESC = FunctionDescriptor.ofVoid(
            JAVA_INT, ADDRESS, JAVA_DOUBLE, JAVA_DOUBLE, JAVA_DOUBLE, ADDRESS);

    private final Arena arena = Arena.ofConfined();
    private final MemorySegment graph;
    private final int nVertices;
    private IterationListener listener;
    private Throwable listenerError;

    /** Sparky.java:124-184: dedupe, adjacency, N, dangling set -- on the GPU. dst[i] == -1: a record without links. */
    public PageRankHip(int device, int nVertices, int[] src, int[] dst, int flags) throws Throwable {
        if (src.length != dst.length) throw new IllegalArgumentException("src and dst lengths differ");
        this.nVertices = nVertices;
        try (Arena call = Arena.ofConfined()) {
            MemorySegment s = call.allocateFrom(JAVA_INT, src);
            MemorySegment d = call.allocateFrom(JAVA_INT, dst);
            MemorySegment out = call.allocate(ADDRESS);
            check((int) CREATE.invokeExact(device, nVertices, (long) src.length, s, d, flags | PR_NO_CANONICAL, out));
            graph = out.get(ADDRESS, 0);
        }
    }

    /** info[i] of pr_graph_info (PR_INFO_* indices). */
    public long[] info() throws Throwable {
        try (Arena call = Arena.ofConfined()) {
            MemorySegment a = call.allocate(JAVA_LONG, PR_INFO_COUNT);
            check((int) INFO.invokeExact(graph, a, PR_INFO_COUNT));
            return a.toArray(JAVA_LONG);
        }
    }

    /** Sparky.java:164-238: init (1.0, or initRanks), then the iterations; returns the final ranks. */
    public double[] run(int iterations, double[] initRanks, IterationListener l, boolean ranksInCallback)
            throws Throwable {
        if (initRanks != null && initRanks.length != nVertices)
            throw new IllegalArgumentException("initRanks must hold " + nVertices + " ranks");
        listener = l;
        listenerError = null;
        try (Arena call = Arena.ofConfined()) {
            MemorySegment init = initRanks == null ? MemorySegment.NULL : call.allocateFrom(JAVA_DOUBLE, initRanks);
            MemorySegment out = call.allocate(JAVA_DOUBLE, Math.max(nVertices, 1));
            MemorySegment cb = MemorySegment.NULL;
            if (l != null) {
                MethodHandle target = MethodHandles.lookup().findVirtual(PageRankHip.class, "upcall",
                        MethodType.methodType(void.class, int.class, MemorySegment.class, double.class,
                                double.class, double.class, MemorySegment.class)).bindTo(this);
                cb = LINKER.upcallStub(target, CB_DESC, call);
            }
            int rc = (int) RUN.invokeExact(graph, iterations, 0.15, 0.85, init, out, cb,
                    ranksInCallback ? PR_CB_RANKS : 0, MemorySegment.NULL);
            if (listenerError != null) throw listenerError;  // an upcall must not unwind into C
            check(rc);
            return out.asSlice(0, 8L * nVertices).toArray(JAVA_DOUBLE);
        } finally {
            listener = null;
        }
    }

    private void upcall(int iter, MemorySegment ranks, double dc, double l1, double ms, MemorySegment user) {
        if (listenerError != null) return;
        try {
            double[] r = ranks.equals(MemorySegment.NULL) ? null
                    : ranks.reinterpret(8L * nVertices).toArray(JAVA_DOUBLE);
            listener.onIteration(iter, r, dc, l1, ms);
        } catch (Throwable t) {
            listenerError = t;
        }
    }

    private static void check(int rc) throws Throwable {
        if (rc != 0) {
            MemorySegment msg = (MemorySegment) LAST_ERROR.invokeExact();
            throw new RuntimeException("libpagerank_hip error " + rc + ": " + msg.reinterpret(4096).getString(0));
        }
    }

    @Override
    public void close() throws Throwable {
        DESTROY.invokeExact(graph);
        arena.close();
    }
}
