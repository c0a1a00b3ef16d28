/*
 * An IByteBufferAllocator (IByteBufferAllocator.java:38-149) whose buffers are
 * pinned host memory from libwsgpu's pool (wsg_host_alloc / wsg_host_release:
 * power-of-two size classes, recycled on release), so socket reads land in memory
 * the H2D copy of a batch reads at full PCIe rate.  The capacity policy
 * (ensureSome / ensure / reduce / extend) is DefaultAllocator's; only the
 * allocation and the release change.  Installed through the session structure
 * factory (ISessionStructureFactory.getAllocator).
 */
package org.snf4j.websocket.gpu;

import java.nio.ByteBuffer;

import org.snf4j.core.allocator.DefaultAllocator;

public class PinnedByteBufferAllocator extends DefaultAllocator {

	public PinnedByteBufferAllocator() {
		super(true);
	}

	@Override
	public boolean isReleasable() {
		return true;
	}

	@Override
	public void release(ByteBuffer buffer) {
		if (buffer != null && buffer.isDirect())
			Wsg.releasePinned(buffer);
	}

	@Override
	protected ByteBuffer allocate(int capacity, boolean direct) {
		if (!direct)
			return super.allocate(capacity, false);
		ByteBuffer b = Wsg.allocPinned(capacity);
		if (b == null)
			throw new OutOfMemoryError("wsg_host_alloc(" + capacity + ")");
		// exactly the requested capacity: DefaultAllocator decides everything from capacity()
		// (a power-of-two class capacity would make reduce() reallocate on every call).  A slice
		// from position 0 keeps the pool buffer's address, which release() looks up.
		b.limit(capacity);
		return b.slice();
	}

	/** The replaced buffer goes back to the pool once its bytes are copied. */
	@Override
	protected ByteBuffer allocateEmpty(int capacity, ByteBuffer buffer) {
		ByteBuffer b = allocate(capacity, buffer.isDirect());
		release(buffer);
		return b;
	}

	@Override
	protected ByteBuffer allocate(int capacity, ByteBuffer buffer) {
		ByteBuffer b = super.allocate(capacity, buffer);
		release(buffer);
		return b;
	}
}
