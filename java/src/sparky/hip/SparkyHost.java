// Host logic of the Sparky-compatible Java drivers (SURVEY.md §8 f2), shared by the FFM driver
// (SparkyHip, JDK 22+) and the JNI driver (SparkyJni, JDK 8..21).  Java 8 syntax and APIs only,
// no java.lang.foreign: it compiles with `javac --release 8` (java/Makefile, tests/test_java_host.py).
//
// Contract (the same as the C++ `pagerank` CLI and `python -m sparky_hip`):
//   * input: "src dst" per line; a single token "src" is a record without 'a' links
//     (Sparky.java:114-118); URLs are interned here, in Java, to dense int IDs in first-appearance
//     order (src before dst) -- the IDs libpagerank_hip takes;
//   * stdout: "Starting iter<i>" before every iteration (Sparky.java:188), then
//     "<url> has rank: <r>." per URL (north_star);
//   * --out DIR: DIR/PageRank<i>/part-00000 with "(url,rank)" lines + _SUCCESS
//     (Sparky.java:237 saveAsTextFile), rank printed by the running JVM's own Double.toString;
//   * --resume: start from a saved PageRank<i> and continue the loop (iterations i+1 .. N-1).
package sparky.hip;

import java.io.BufferedReader;
import java.io.BufferedWriter;
import java.io.IOException;
import java.io.PrintStream;
import java.nio.charset.StandardCharsets;
import java.nio.file.DirectoryStream;
import java.nio.file.Files;
import java.nio.file.Path;
import java.nio.file.Paths;
import java.util.ArrayList;
import java.util.Arrays;
import java.util.Collections;
import java.util.HashMap;
import java.util.List;
import java.util.Map;
import java.util.regex.Matcher;
import java.util.regex.Pattern;

public final class SparkyHost {
    private SparkyHost() {}

    /** One binding of libpagerank_hip: build the graph, run the iterations (Sparky.java:124-238). */
    public interface Engine {
        double[] run(int device, int nVertices, int[] src, int[] dst, int flags, int iterations, double[] initRanks,
                     IterationListener listener, boolean ranksInCallback) throws Throwable;
    }

    /** First-appearance interning of the edge list (src before dst). */
    static final class Edges {
        final Map<String, Integer> ids = new HashMap<String, Integer>();
        final List<String> urls = new ArrayList<String>();
        int[] src = new int[1024], dst = new int[1024];
        int n;

        int intern(String u) {
            Integer id = ids.get(u);
            if (id == null) {
                id = urls.size();
                ids.put(u, id);
                urls.add(u);
            }
            return id;
        }

        void add(int s, int d) {
            if (n == src.length) {
                src = Arrays.copyOf(src, 2 * n);
                dst = Arrays.copyOf(dst, 2 * n);
            }
            src[n] = s;
            dst[n++] = d;
        }

        static Edges read(Path p) throws IOException {
            Edges e = new Edges();
            BufferedReader r = Files.newBufferedReader(p, StandardCharsets.UTF_8);
            try {
                String line;
                int ln = 0;
                while ((line = r.readLine()) != null) {
                    ++ln;
                    String t = line.trim();
                    if (t.isEmpty()) continue;
                    String[] tok = t.split("[ \t]+");
                    if (tok.length > 2)
                        throw new IOException("line " + ln + ": expected 'src [dst]', got " + tok.length + " tokens");
                    int s = e.intern(tok[0]);
                    e.add(s, tok.length == 2 ? e.intern(tok[1]) : -1);
                }
            } finally {
                r.close();
            }
            return e;
        }
    }

    static void writePart(Path out, int iter, List<String> urls, double[] ranks) throws IOException {
        Path d = out.resolve("PageRank" + iter);
        Files.createDirectories(d);
        BufferedWriter w = Files.newBufferedWriter(d.resolve("part-00000"), StandardCharsets.UTF_8);
        try {
            for (int v = 0; v < urls.size(); ++v) w.write("(" + urls.get(v) + "," + Double.toString(ranks[v]) + ")\n");
        } finally {
            w.close();
        }
        Files.write(d.resolve("_SUCCESS"), new byte[0]);
    }

    static double[] readSaved(Path dir, Edges e) throws IOException {
        double[] r = new double[e.urls.size()];
        boolean[] seen = new boolean[r.length];
        int nSeen = 0;
        List<Path> parts = new ArrayList<Path>();
        DirectoryStream<Path> ds = Files.newDirectoryStream(dir, "part-*");
        try {
            for (Path p : ds) parts.add(p);
        } finally {
            ds.close();
        }
        if (parts.isEmpty()) throw new IOException("no part-* files in " + dir);
        Collections.sort(parts);
        for (Path p : parts) {
            for (String line : Files.readAllLines(p, StandardCharsets.UTF_8)) {
                if (line.isEmpty()) continue;
                if (!line.startsWith("(") || !line.endsWith(")")) throw new IOException(p + ": expected '(url,rank)'");
                String body = line.substring(1, line.length() - 1);
                int c = body.lastIndexOf(',');  // URLs may hold commas; the rank never does
                Integer id = c < 0 ? null : e.ids.get(body.substring(0, c));
                if (id == null) throw new IOException(p + ": URL not in the edge list: " + line);
                if (seen[id]) throw new IOException(p + ": URL listed twice: " + line);
                seen[id] = true;
                ++nSeen;
                r[id] = Double.parseDouble(body.substring(c + 1));
            }
        }
        if (nSeen != r.length) throw new IOException(dir + ": " + (r.length - nSeen) + " URL(s) have no saved rank");
        return r;
    }

    /** The driver: parse args, intern, run through `engine`, write the outputs. */
    public static void main(String[] args, Engine engine) throws Throwable {
        String path = null, out = null, resume = null;
        int iterations = 10, device = 0, flags = 0, pos = 0;  // flags: PR_DANGLING_LOCAL
        boolean saveEvery = false, quiet = false;
        for (int i = 0; i < args.length; ++i) {
            String a = args[i];
            if (a.equals("--out")) out = args[++i];
            else if (a.equals("--save-every-iter")) saveEvery = true;
            else if (a.equals("--quiet")) quiet = true;
            else if (a.equals("--dangling=local")) flags = 0;
            else if (a.equals("--dangling=none")) flags = 1;  // PR_DANGLING_NONE
            else if (a.equals("--device")) device = Integer.parseInt(args[++i]);
            else if (a.equals("--resume")) resume = args[++i];
            else if (a.startsWith("-")) throw new IllegalArgumentException("unknown option " + a);
            else if (pos++ == 0) path = a;
            else iterations = Integer.parseInt(a);  // Sparky.java:187
        }
        if (path == null) throw new IllegalArgumentException("usage: <driver> <edge-list> [iterations=10] [options]");
        final Edges e = Edges.read(Paths.get(path));
        double[] init = null;
        int start = 0;
        if (resume != null) {
            init = readSaved(Paths.get(resume), e);
            Matcher m = Pattern.compile("PageRank(\\d+)/*$").matcher(resume);
            start = m.find() ? Integer.parseInt(m.group(1)) + 1 : 0;
        }
        final int first = start, total = iterations;
        final String outDir = out;
        final boolean every = saveEvery;
        final PrintStream so = System.out;
        int nRun = Math.max(total - first, 0);
        if (nRun > 0) so.println("Starting iter" + first);
        IterationListener listener = new IterationListener() {
            @Override
            public void onIteration(int itRun, double[] r, double dc, double l1, double ms) {
                int it = first + itRun;
                try {
                    if (outDir != null && (every || it == total - 1)) writePart(Paths.get(outDir), it, e.urls, r);
                } catch (IOException ex) {
                    throw new RuntimeException(ex);
                }
                if (it + 1 < total) so.println("Starting iter" + (it + 1));
            }
        };
        double[] ranks = engine.run(device, e.urls.size(), Arrays.copyOf(e.src, e.n), Arrays.copyOf(e.dst, e.n), flags,
                nRun, init, listener, outDir != null);
        if (!quiet)
            for (int v = 0; v < e.urls.size(); ++v) so.println(e.urls.get(v) + " has rank: " + Double.toString(ranks[v]) + ".");
        so.flush();
    }
}
