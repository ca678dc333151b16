// Per-iteration hook of both Java bindings (FFM: PageRankHip, JNI: PageRankJni).  Java 8 syntax and
// no java.lang.foreign, so the JNI path compiles on JDK 8..21.
package sparky.hip;

/** ranks is null unless requested (original-ID order, V doubles); Sparky.java:188, :237 run here. */
public interface IterationListener {
    void onIteration(int iteration, double[] ranks, double danglingSum, double l1Delta, double ms);
}
